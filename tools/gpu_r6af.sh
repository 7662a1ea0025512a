#!/bin/bash
# r6 call AF: staging-pool threads (2 / 4 / 8) with the final JPEG path, 51,200-distinct pass, interleaved twice.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_af
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for t in 4 2 8; do
    DML_STAGING_THREADS=$t timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/distinct_t${t}_r$r.log 2>&1 || { tail -20 $O/distinct_t${t}_r$r.log; exit 1; }
    echo "threads=$t r$r $(python tools/bench_summary.py $O/distinct_t${t}_r$r.log | sed 's/.*ResNet50 [0-9]*//')"
  done
done
