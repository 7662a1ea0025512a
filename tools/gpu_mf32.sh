#!/bin/bash
# 16x16x32 vs 32x32x16 MFMA tiles: numerics of the MF 32 configs (48..55), then
# every ResNet50 / InceptionV3 conv shape timed on each MF 16 tile and its MF 32
# twin (conv_bench.py, one process, same buffers). Each GPU step has its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "test_conv_matches_fp32 or test_conv_subsampled_residual" > gpurun_out/pytest_mf32.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_mf32.log; [ $rc -eq 0 ] || exit $rc
# r2_v23 measured 8 pairs (14/48 15/49 11/50 32/51 30/52 31/53 26/54 23/55); 48 and 49 are kept
PAIRS=14,48,15,49
timeout -k 10 600 python -u tools/conv_bench.py --model ResNet50 --batch 128 --cfgs $PAIRS --out gpurun_out/mf32_r50.json \
  > gpurun_out/mf32_r50.log 2>&1 && tail -1 gpurun_out/mf32_r50.log || { tail -20 gpurun_out/mf32_r50.log; exit 1; }
timeout -k 10 600 python -u tools/conv_bench.py --model InceptionV3 --batch 64 --cfgs $PAIRS --out gpurun_out/mf32_inc.json \
  > gpurun_out/mf32_inc.log 2>&1 && tail -1 gpurun_out/mf32_inc.log || { tail -20 gpurun_out/mf32_inc.log; exit 1; }
