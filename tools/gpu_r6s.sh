#!/bin/bash
# r6 call S: the 51,200-distinct pass at image-staging look-ahead 8 (default) / 16 / 24, interleaved twice.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_s
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for d in 8 16 24; do
    DML_STAGE_DEPTH=$d timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/distinct_d${d}_r$r.log 2>&1 || { tail -20 $O/distinct_d${d}_r$r.log; exit 1; }
    echo "depth=$d r$r $(python tools/bench_summary.py $O/distinct_d${d}_r$r.log | sed 's/.*store-images//')"
  done
done
