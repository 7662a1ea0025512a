#!/bin/bash
# CU-masked sub-batch streams (parallel/cu_mask.py): where masked blocks run
# (tools/cu_mask_probe.py), then the bench (both models) per DML_CU_MASK pattern.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/cu_mask_probe.py --out gpurun_out/cu_mask_probe.json > gpurun_out/cu_mask_probe.log 2>&1 \
  && tail -25 gpurun_out/cu_mask_probe.log || { tail -20 gpurun_out/cu_mask_probe.log; exit 1; }
for pat in none ${PATTERNS:-lohi mod8 evenodd}; do
  if [ "$pat" = none ]; then unset DML_CU_MASK; else export DML_CU_MASK=$pat; fi
  timeout -k 10 600 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_cm_$pat.log 2>&1 \
    && echo "$pat: $(tail -1 gpurun_out/bench_cm_$pat.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["models"]["InceptionV3"]["value"], d["verified_top5"])')" \
    || { tail -20 gpurun_out/bench_cm_$pat.log; exit 1; }
done
