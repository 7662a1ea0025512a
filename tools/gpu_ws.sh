#!/bin/bash
# One gpurun call for the warp-specialised conv tiles: numerics tests (fp32 reference and
# bit-identity with the v2 tiles), then the per-shape cold A/B against the v2 tiles.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_ws_gpu.py -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/ws_pytest.log 2>&1; rc=$?
tail -8 gpurun_out/ws_pytest.log
# a test failure (1) still allows the timing pass; a timeout / crash does not
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u tools/conv_ws_ab.py ${AB_ARGS:-} --out gpurun_out/ws_ab.json > gpurun_out/ws_ab.log 2>&1; rc2=$?
cat gpurun_out/ws_ab.log | grep -v "^    " | tail -40
exit $(( rc > rc2 ? rc : rc2 ))
