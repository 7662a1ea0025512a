#!/bin/bash
# r6 call AE: a window's GPU decode launched in one native call (dml_jpeg_launch): JPEG + store
# path GPU tests, the window bench, the 51,200-distinct pass twice.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_ae
mkdir -p $O
export TMPDIR=/tmp
true

timeout -k 10 120 python tools/jpeg_bench.py > $O/jpeg_bench.log 2>&1 || { tail -5 $O/jpeg_bench.log; exit 1; }
grep -h window $O/jpeg_bench.log | tr '\n' ' '; echo
for r in 1 2 3; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/distinct_r$r.log 2>&1 || { tail -20 $O/distinct_r$r.log; exit 1; }
  python tools/bench_summary.py $O/distinct_r$r.log
  grep -o '"loop_phase_s": {[^}]*}' $O/distinct_r$r.log | tail -1
done
