#!/bin/bash
# The lagged result gather's own cost on one GPU (bench.py --gather-lag 1 vs 0), interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for l in 0 1; do
    for m in ResNet50 InceptionV3; do
      timeout -k 10 300 python -u bench.py --model $m --steps 30 --warmup 5 --no-service --gather-lag $l \
        > gpurun_out/lag_${l}_${m}_$r.log 2>&1 || { tail -20 gpurun_out/lag_${l}_${m}_$r.log; exit 1; }
      echo "lag $l $m round $r: $(grep '"metric"' gpurun_out/lag_${l}_${m}_$r.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["p50_latency_ms"], r["verified_top5"])')"
    done
  done
done
