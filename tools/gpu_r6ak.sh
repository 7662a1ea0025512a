#!/bin/bash
# r6 call AK: GPU JPEG side streams (2 default / 1) in the 51,200-distinct pass, interleaved twice.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_ak
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in 2 1; do
    DML_JPEG_STREAMS=$v timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/distinct_s${v}_r$r.log 2>&1 || { tail -20 $O/distinct_s${v}_r$r.log; exit 1; }
    echo "streams=$v r$r $(python tools/bench_summary.py $O/distinct_s${v}_r$r.log | sed 's/.*ResNet50 [0-9]*//')"
  done
done
