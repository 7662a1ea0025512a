#!/bin/bash
# Block-order twins (cfg 62 = 14, 63 = 11 with pixel tiles fastest): numerics,
# then the stage-4/5 ResNet50 shapes warm and cold (--flush).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "test_conv_matches_fp32 or test_conv_subsampled_residual" > gpurun_out/pytest_ord.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_ord.log; [ $rc -eq 0 ] || exit $rc
for m in warm flush; do
  F=""; [ $m = flush ] && F="--flush"
  timeout -k 10 600 python -u tools/conv_bench.py --model ResNet50 --batch 128 $F --only conv4,conv5 --cfgs 14,62,11,63 \
    --out gpurun_out/ord_$m.json > gpurun_out/ord_$m.log 2>&1 && tail -1 gpurun_out/ord_$m.log || { tail -20 gpurun_out/ord_$m.log; exit 1; }
done
