#!/bin/bash
# Run-to-run spread of the headline bench on one box: N back-to-back runs.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in $(seq 1 ${N:-5}); do
  timeout -k 10 600 python bench.py --steps 30 --warmup 5 > gpurun_out/rep_$i.log 2>&1 \
    && echo "run $i: $(tail -1 gpurun_out/rep_$i.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["models"]["InceptionV3"]["value"], d["p50_latency_ms"], d["verified_top5"])')" \
    || { tail -20 gpurun_out/rep_$i.log; exit 1; }
done
