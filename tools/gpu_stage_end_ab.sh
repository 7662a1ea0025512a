#!/bin/bash
# Stage-3-end chained boundary (DML_CHAIN_STAGE_END=2): numerics, then interleaved pipeline A/B.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py -k "stage_end" -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_se3.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_se3.log; [ $rc -eq 0 ] || exit $rc
DML_CHAIN_STAGE_END=2 timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py -k "fused_blocks_equal and 256-1-1" -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_se3_engine.log 2>&1; tail -2 gpurun_out/pytest_se3_engine.log
VARIANTS="-;DML_CHAIN_STAGE_END=2" ROUNDS=3 BENCH_ARGS="--models ResNet50 --no-service" bash tools/gpu_env_ab.sh
