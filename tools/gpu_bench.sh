#!/bin/bash
# Pipeline check: serving-pipeline GPU test, then the bench (both models), then a
# rocprofv3 kernel trace of a short bench for the GPU-idle-gap analysis.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_serving_gpu.py > gpurun_out/pytest_pipe.log 2>&1 || { tail -30 gpurun_out/pytest_pipe.log; exit 1; }
tail -1 gpurun_out/pytest_pipe.log
timeout -k 10 600 python bench.py --steps 30 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log || { tail -30 gpurun_out/bench.log; exit 1; }
if [ -n "$PROFILE" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 2 --models ResNet50 > $GRAFT_REPO_ROOT/gpurun_out/prof2.log 2>&1 && echo profiled || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof2.log; exit 1; }
fi
