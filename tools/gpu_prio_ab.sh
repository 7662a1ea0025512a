#!/bin/bash
# Sub-batch stream priority A/B (DML_SPLIT_STREAM_PRIO), interleaved rounds, both models.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for p in none -1 1; do
    for m in ResNet50 InceptionV3; do
      if [ "$p" = none ]; then unset DML_SPLIT_STREAM_PRIO; else export DML_SPLIT_STREAM_PRIO=$p; fi
      timeout -k 10 300 python -u bench.py --model $m --steps 30 --warmup 5 --no-service \
        > gpurun_out/prio_${p}_${m}_$r.log 2>&1 || { tail -20 gpurun_out/prio_${p}_${m}_$r.log; exit 1; }
      echo "prio $p $m round $r: $(grep '"metric"' gpurun_out/prio_${p}_${m}_$r.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
    done
  done
done
