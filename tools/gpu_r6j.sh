#!/bin/bash
# r6 call J: the world-8 output-path capacity harness (CPU processes) with the result collect
# on and off, interleaved, twice (the margin with the gather in the path).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6_collect
export TMPDIR=/tmp
for round in 1 2; do
  for c in 1 0; do
    DML_COLLECT_RESULTS=$c timeout -k 10 240 python tools/store_capacity.py --world 8 --rate 600 --batches-per-rank 600 \
      --out gpurun_out/r6_collect/cap_c${c}_r${round}.json > gpurun_out/r6_collect/cap_c${c}_r${round}.log 2>&1 || { tail -20 gpurun_out/r6_collect/cap_c${c}_r${round}.log; exit 1; }
    echo "collect=$c round=$round"; grep -E '^\{"world"|CAPACITY' gpurun_out/r6_collect/cap_c${c}_r${round}.log | cut -c1-220
  done
done
