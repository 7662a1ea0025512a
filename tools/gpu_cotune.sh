#!/bin/bash
# Pipeline co-tuning pass (tools/cotune_pipe.py) over MODEL (default InceptionV3) with CANDS candidates per op.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/cotune_pipe.py --model ${MODEL:-InceptionV3} --cands ${CANDS:-4} --budget_s ${BUDGET:-540} \
  --out gpurun_out/cotune2_${MODEL:-InceptionV3}.json > gpurun_out/cotune2_${MODEL:-InceptionV3}.log 2>&1 || { tail -20 gpurun_out/cotune2_${MODEL:-InceptionV3}.log; exit 1; }
tail -1 gpurun_out/cotune2_${MODEL:-InceptionV3}.log | cut -c1-600
