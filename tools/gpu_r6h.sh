#!/bin/bash
# r6 call H: sub-batch phase-shift A/B (DML_PHASE_SHIFT_US: the extra stream starts this much
# behind), 200 timed steps, interleaved, both models.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for m in InceptionV3 ResNet50; do
    for sh in 0 450 900 1300; do
      DML_PHASE_SHIFT_US=$sh timeout -k 10 300 python bench.py --model $m --no-service --steps 200 --warmup 5 > gpurun_out/ph_${m}_${sh}_r$r.log 2>&1 || { tail -20 gpurun_out/ph_${m}_${sh}_r$r.log; exit 1; }
      echo "r$r $m shift=$sh $(grep -o '"value": [0-9.]*' gpurun_out/ph_${m}_${sh}_r$r.log | head -1) $(grep -o '"verified_top5": [a-z]*' gpurun_out/ph_${m}_${sh}_r$r.log | head -1)"
    done
  done
done
