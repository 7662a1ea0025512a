#!/bin/bash
# Fused-boundary GPU tests, then pipeline co-tuning (tools/cotune_pipe.py) of both models on the
# current defaults; the tuning table after the run is copied to gpurun_out/.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_stem_gpu.py -k "fused_blocks or stem" -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_blocks.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_blocks.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --models ResNet50 --no-service --steps 60 > gpurun_out/bench_r50.log 2>&1 &&
  echo "bench: $(tail -1 gpurun_out/bench_r50.log | grep -o '"value": [0-9.]*' | head -1)" || exit 1
for m in ResNet50 InceptionV3; do
  timeout -k 10 700 python -u tools/cotune_pipe.py --model $m --budget_s 420 --out gpurun_out/cotune_$m.json \
    > gpurun_out/cotune_$m.log 2>&1 || { tail -20 gpurun_out/cotune_$m.log; exit 1; }
  tail -1 gpurun_out/cotune_$m.log | cut -c1-400
done
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/conv_tuning.json
