#!/bin/bash
# Late-residual twins (cfg 56..60): numerics, a base-vs-twin timing of the
# ResNet50 residual shapes, then both model benches (the tuner re-times every
# residual conv against the enlarged candidate set; the table is copied out).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "test_conv_matches_fp32 or test_conv_subsampled_residual" > gpurun_out/pytest_late.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_late.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/conv_bench.py --model ResNet50 --batch 128 --only _3_conv \
  --cfgs 30,56,31,57,25,58,28,59,23,60,11,14,15,26,27 --out gpurun_out/late_r50.json \
  > gpurun_out/late_r50.log 2>&1 && tail -1 gpurun_out/late_r50.log || { tail -20 gpurun_out/late_r50.log; exit 1; }
timeout -k 10 900 python bench.py --steps 20 --warmup 5 --op-times gpurun_out/op_times.json > gpurun_out/bench.log 2>&1 \
  && tail -1 gpurun_out/bench.log || { tail -30 gpurun_out/bench.log; exit 1; }
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench2.log 2>&1 && tail -1 gpurun_out/bench2.log
