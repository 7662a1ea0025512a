#!/bin/bash
# One gpurun call for the r5 conv tiles: numerics of the patch-stationary (140..143) and the
# warp-specialised / persistent / fragment-prefetch tiles, the per-shape cold A/B of all of
# them against v2 (tools/conv_ws_ab.py), (TUNE=1) tuning-table adoption of the new ids with an
# interleaved bench A/B, the full bench (service + store-image pass) and (STORECAP=1) the
# world-8 output-store capacity harness. Each GPU step has its own limit; a failure ends the call.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_pt_gpu.py tests/test_conv_ws_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r5_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/conv_ws_ab.py --out gpurun_out/ws_ab_all.json > gpurun_out/ws_ab_all.log 2>&1 || { tail -20 gpurun_out/ws_ab_all.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ws_ab_all.log | grep -v "^    "
if [ -n "$TUNE" ]; then
  ADD=113,114,115,116,117,118,140,141,142,143,144,145,146 bash tools/gpu_ws_tune.sh || exit 1
fi
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
python tools/bench_summary.py gpurun_out/bench_full.log
if [ -n "$STORECAP" ]; then
  timeout -k 10 600 python -u tools/store_capacity.py --world 8 --rate 370 --batches-per-rank 300 --out gpurun_out/store_capacity_box3.json > gpurun_out/store_capacity_box3.log 2>&1; echo "storecap rc=$?"; grep world gpurun_out/store_capacity_box3.log | cut -c1-700
fi
