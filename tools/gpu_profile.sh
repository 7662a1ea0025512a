#!/bin/bash
# One gpurun call: GPU tests of the kernels, bench with per-op times for both models (the
# roofline CSVs), a rocprofv3 kernel-stats profile of the ResNet50 bench, store capacity.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/prof_r5
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --op-times gpurun_out/op_times_r50.json > gpurun_out/bench_r50.log 2>&1 || { tail -30 gpurun_out/bench_r50.log; exit 1; }
python tools/bench_summary.py gpurun_out/bench_r50.log
timeout -k 10 600 python -u bench.py --model InceptionV3 --steps 20 --warmup 5 --no-service --op-times gpurun_out/op_times_inc.json > gpurun_out/bench_inc.log 2>&1 || { tail -30 gpurun_out/bench_inc.log; exit 1; }
python tools/bench_summary.py gpurun_out/bench_inc.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-service > $GRAFT_REPO_ROOT/gpurun_out/prof_r5.log 2>&1 && echo profiled || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_r5.log; exit 1; }
cd $GRAFT_REPO_ROOT
if [ -n "$STORECAP" ]; then
  timeout -k 10 600 python -u tools/store_capacity.py --world 8 --rate 370 --batches-per-rank 300 --out gpurun_out/store_capacity_box2.json > gpurun_out/store_capacity_box2.log 2>&1; echo "storecap rc=$?"; grep world gpurun_out/store_capacity_box2.log | cut -c1-300
fi
