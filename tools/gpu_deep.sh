#!/bin/bash
# Deep BK64 rings: kernel numerics on every conv class, per-shape times on the
# long-K layers, then both models' bench with a fresh tuning table (new tag).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/deep
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "matches_fp32 or refused" > gpurun_out/deep/pytest.log 2>&1 || { tail -40 gpurun_out/deep/pytest.log; exit 1; }
tail -1 gpurun_out/deep/pytest.log
timeout -k 10 300 python tools/conv_bench.py --model ResNet50 --batch 128 --only conv4,conv5 \
  --cfgs 11,14,22,29,30,31,32,33,40,41,42,43,44 --out gpurun_out/deep/cb_r50.json > gpurun_out/deep/cb_r50.log 2>&1 \
  && tail -1 gpurun_out/deep/cb_r50.log || { tail -20 gpurun_out/deep/cb_r50.log; exit 1; }
timeout -k 10 300 python tools/conv_bench.py --model InceptionV3 --batch 64 --only conv2d_8,conv2d_9 \
  --cfgs 11,14,22,29,30,31,32,33,40,41,42,43,44 --out gpurun_out/deep/cb_inc.json > gpurun_out/deep/cb_inc.log 2>&1 \
  && tail -1 gpurun_out/deep/cb_inc.log || { tail -20 gpurun_out/deep/cb_inc.log; exit 1; }
timeout -k 10 900 python bench.py --steps 30 --warmup 5 > gpurun_out/deep/bench.log 2>&1 \
  && tail -1 gpurun_out/deep/bench.log | cut -c1-200 || { tail -30 gpurun_out/deep/bench.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/deep/bench.log").read().strip().splitlines()[-1])
print("ResNet50", d["value"], "InceptionV3", d["models"]["InceptionV3"]["value"])
PY
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/deep/conv_tuning.json
