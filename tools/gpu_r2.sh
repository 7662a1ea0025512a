#!/bin/bash
# Round-2 GPU verification: new serving-path GPU tests first, then the whole GPU
# suite, smoke, the bench (ResNet50 headline + InceptionV3 sub-record) and the
# concurrent collective-service bench at world 1. Each step has its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_serving_gpu.py tests/test_engine_gpu.py -k "matches_oracle" > gpurun_out/pytest_new.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|rel err" gpurun_out/pytest_new.log | tail -20; [ $rc -eq 0 ] || exit $rc
if [ -z "$QUICK" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log || { tail -30 gpurun_out/bench.log; exit 1; }
timeout -k 10 600 python tools/serve_bench.py --resnet-images 20480 --inception-images 10240 > gpurun_out/serve_bench.log 2>&1 && tail -1 gpurun_out/serve_bench.log || { tail -30 gpurun_out/serve_bench.log; exit 1; }
