#!/bin/bash
# r6 call Y: serving-engine stream priority (DML_SERVE_STREAM_PRIO 0 / -1) in the
# 51,200-distinct pass, where the model shares the GPU with the JPEG decodes; interleaved twice.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_y
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in 0 -1; do
    DML_SERVE_STREAM_PRIO=$v timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/distinct_p${v}_r$r.log 2>&1 || { tail -20 $O/distinct_p${v}_r$r.log; exit 1; }
    echo "prio=$v r$r $(python tools/bench_summary.py $O/distinct_p${v}_r$r.log | sed 's/.*ResNet50 [0-9]*//')"
  done
done
