#!/bin/bash
# Tile tables tuned after a dirty (default, c5cold) vs a clean (DML_TUNE_SCRUB=clean, c6clean)
# L2/MALL eviction, end to end, interleaved; the clean table is tuned by its first run.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for m in ResNet50 InceptionV3; do
    for sc in dirty clean; do
      log=gpurun_out/scrub_${sc}_${m}_$r.log
      DML_TUNE_SCRUB=$sc DML_TUNING_CACHE=$([ $sc = clean ] && echo gpurun_out/conv_tuning_clean.json || echo distributed_machine_learning_amd/tuning/conv_tuning.json) \
        timeout -k 10 400 python -u bench.py --model $m --steps 30 --warmup 5 --no-service > $log 2>&1 || { tail -20 $log; exit 1; }
      echo "$sc $m round $r: $(grep '"metric"' $log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["verified_top5"])')"
    done
  done
done
