#!/bin/bash
# r3: the 3-stage BK64 64-channel tiles (cfg 38 / 39) against the tuned ones, cold caches, on the
# layers that run the 2-stage 128x64 tile (cfg 15) today; plus their numerics tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "cfg38 or cfg39 or 38 or 39" -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_tile38.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_tile38.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/conv_bench.py --model ResNet50 --batch 128 --flush --cfgs 12,15,27,38,39 \
  --only conv2_block1_2,conv2_block2_2 --out gpurun_out/cb38_r50.json > gpurun_out/cb38_r50.log 2>&1 || { tail -20 gpurun_out/cb38_r50.log; exit 1; }
timeout -k 10 500 python tools/conv_bench.py --model InceptionV3 --batch 64 --flush --cfgs 14,15,27,38,39 \
  --only conv2d_5,conv2d_11,conv2d_30,conv2d_39,conv2d_48,conv2d_68,conv2d_75 --out gpurun_out/cb38_inc.json \
  > gpurun_out/cb38_inc.log 2>&1 || { tail -20 gpurun_out/cb38_inc.log; exit 1; }
tail -30 gpurun_out/cb38_r50.log; tail -40 gpurun_out/cb38_inc.log
