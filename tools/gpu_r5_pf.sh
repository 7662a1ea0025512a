#!/bin/bash
# One gpurun call: the fragment-prefetch warp-specialised tiles (cfg 113..118) — numerics
# tests of every ws/wsp tile, per-shape cold A/B, tuning-table adoption of the PF tiles with
# an interleaved bench A/B (tools/gpu_ws_tune.sh), then the full bench (service + the
# store-image pass) and (STORECAP=1) the world-8 output-store capacity harness.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_ws_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ws_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/ws_pytest.log
[ $rc -eq 0 ] || exit $rc
WS=100,101,102,103,104,105,106,107,108,109,110,111,112,113,114,115,116,117,118,120,121,122,123,124,125,126,127,128,129
timeout -k 10 900 python -u tools/conv_ws_ab.py --ws $WS --out gpurun_out/ws_ab_pf.json > gpurun_out/ws_ab_pf.log 2>&1 || { tail -20 gpurun_out/ws_ab_pf.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ws_ab_pf.log
if [ -n "$TUNE" ]; then
  ADD=113,114,115,116,117,118 bash tools/gpu_ws_tune.sh || exit 1
fi
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
python tools/bench_summary.py gpurun_out/bench_full.log
if [ -n "$STORECAP" ]; then
  timeout -k 10 600 python -u tools/store_capacity.py --world 8 --rate 370 --batches-per-rank 300 --out gpurun_out/store_capacity_box3.json > gpurun_out/store_capacity_box3.log 2>&1; echo "storecap rc=$?"; grep world gpurun_out/store_capacity_box3.log | cut -c1-600
fi
