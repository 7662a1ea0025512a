#!/bin/bash
# One gpurun call: the store-image GPU tests (JPEG decode, resize), the default bench (headline +
# service + store-image pass) and the honest 51,200-distinct-image store pass, then (ADD=<cfg
# ids>) tuning-table adoption with an interleaved bench A/B (tools/gpu_ws_tune.sh).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py tests/test_resize_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/store_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/store_pytest.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/store_pytest.log; exit $rc; }
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
python tools/bench_summary.py gpurun_out/bench_full.log
timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 --svc-store-images 51200 --svc-store-time-limit 600 > gpurun_out/bench_distinct.log 2>&1 || { tail -30 gpurun_out/bench_distinct.log; exit 1; }
python tools/bench_summary.py gpurun_out/bench_distinct.log
if [ -n "$ADD" ]; then
  bash tools/gpu_ws_tune.sh || exit 1
fi
