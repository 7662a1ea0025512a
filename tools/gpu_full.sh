#!/bin/bash
# One gpurun call: the whole GPU suite, the default bench (headline + service + store-image
# pass), the honest distinct-image store pass (51,200 names, every one fetched + decoded once),
# and the world-8 output-store capacity harness (CPU processes). Each step has its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1; rc=$?
tail -15 gpurun_out/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
python tools/bench_summary.py gpurun_out/bench_full.log
if [ -n "$DISTINCT" ]; then
  timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 --svc-store-images 51200 --svc-store-time-limit 600 > gpurun_out/bench_distinct.log 2>&1 || { tail -30 gpurun_out/bench_distinct.log; exit 1; }
  python tools/bench_summary.py gpurun_out/bench_distinct.log
fi
if [ -n "$STORECAP" ]; then
  timeout -k 10 600 python -u tools/store_capacity.py --world 8 --rate 370 --batches-per-rank 1200 --out gpurun_out/store_capacity_box4.json > gpurun_out/store_capacity_box4.log 2>&1; echo "storecap rc=$?"; grep -E "CAPACITY" gpurun_out/store_capacity_box4.log
fi
