#!/bin/bash
# r6 call T: the GPU launcher round trip with get-output from gathered rows, incl. the forced
# one-rank RCCL gather of the result group.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_rank_service_gpu.py -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" $O/pytest.log | tail -8
exit $rc
