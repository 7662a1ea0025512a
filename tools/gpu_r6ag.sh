#!/bin/bash
# r6 call AG: the driver's command with a 1 s (default) vs 3 s clock spin-up, interleaved twice (no service passes).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_ag
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for sp in 1 3; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-service --spinup-s $sp > $O/bench_s${sp}_r$r.log 2>&1 || { tail -20 $O/bench_s${sp}_r$r.log; exit 1; }
    echo "spinup=$sp r$r $(python tools/bench_summary.py $O/bench_s${sp}_r$r.log | sed 's/.*log: //')"
  done
done
