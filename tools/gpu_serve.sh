#!/bin/bash
# Collective-service GPU check: serving-path GPU tests + concurrent serve bench (world 1).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_serving_gpu.py > gpurun_out/pytest_serving.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_serving.log | tail -10; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_serving.log; exit $rc; }
timeout -k 10 600 python tools/serve_bench.py --resnet-images ${RI:-40960} --inception-images ${II:-20480} > gpurun_out/serve_bench.log 2>&1 && tail -1 gpurun_out/serve_bench.log || { tail -30 gpurun_out/serve_bench.log; exit 1; }
