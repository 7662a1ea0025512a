#!/bin/bash
# r6 call N: the 51,200-distinct pass with 32 (default) / 8 / 4 staging-pool threads, interleaved twice.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_n
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for t in 32 8 4; do
    DML_DECODE_THREADS=$t timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/distinct_t${t}_r$r.log 2>&1 || { tail -20 $O/distinct_t${t}_r$r.log; exit 1; }
    echo "threads=$t r$r $(python tools/bench_summary.py $O/distinct_t${t}_r$r.log | sed 's/.*store-images//')"
    grep -o '"loop_phase_s": {[^}]*}' $O/distinct_t${t}_r$r.log | tail -1
  done
done
