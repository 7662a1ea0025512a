#!/bin/bash
# Sub-batch layout A/B for ResNet50 b256 (one box, interleaved rounds): 2 / 4 / 8 sub-batches,
# with HIP's default 4 hardware queues and with 8.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for v in "2 4" "4 4" "4 8" "8 8"; do
    set -- $v
    GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python bench.py --models ResNet50 --no-service --steps 60 --warmup 5 --splits $1 \
      > gpurun_out/splits_$1_q$2_r$r.log 2>&1 || { tail -20 gpurun_out/splits_$1_q$2_r$r.log; exit 1; }
    echo "round $r splits $1 hwq $2: $(tail -1 gpurun_out/splits_$1_q$2_r$r.log | cut -c1-150)"
  done
done
