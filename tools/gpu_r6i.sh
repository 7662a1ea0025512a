#!/bin/bash
# r6 call I: the GPU suite on the tree with the result collect, then the driver's default
# bench command (its service passes carry the get-output A/B record).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/i_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/i_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py > gpurun_out/i_bench.log 2>&1 || { tail -20 gpurun_out/i_bench.log; exit 1; }
python tools/bench_summary.py gpurun_out/i_bench.log
grep -o '"get_output": {[^}]*}[^}]*}[^}]*}[^}]*}' gpurun_out/i_bench.log || true
