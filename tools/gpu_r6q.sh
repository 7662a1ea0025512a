#!/bin/bash
# r6 call Q: the 51,200-distinct pass with the serve loop under cProfile (current tree).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_q
mkdir -p $O
export TMPDIR=/tmp
DML_PROFILE_SERVE=$PWD/$O/serve_profile.txt timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/distinct_prof.log 2>&1 || { tail -20 $O/distinct_prof.log; exit 1; }
python tools/bench_summary.py $O/distinct_prof.log
grep -o '"loop_phase_s": {[^}]*}' $O/distinct_prof.log | tail -1
