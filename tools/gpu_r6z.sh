#!/bin/bash
# r6 call Z: config 4 on one GPU, time-sliced (default) vs the reference's one-model-at-a-time
# split (DML_ONE_RANK_SLICE=0): the service pass of bench.py, interleaved twice.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_z
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in 1 0; do
    DML_ONE_RANK_SLICE=$v timeout -k 10 400 python bench.py --gpus 1 --steps 5 --warmup 2 --models ResNet50 --svc-store-images 0 --kill-pass off > $O/svc_s${v}_r$r.log 2>&1 || { tail -20 $O/svc_s${v}_r$r.log; exit 1; }
    python - <<PY
import json
l = [x for x in open("$O/svc_s${v}_r$r.log") if x.startswith('{"metric"')][-1]
s = json.loads(l)["service"]
print("slice=$v r$r service", s.get("value"), "p50", s.get("p50_latency_ms"), "split", s.get("fair_share_splits"))
PY
  done
done
