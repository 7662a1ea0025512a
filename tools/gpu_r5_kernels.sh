#!/bin/bash
# One gpurun call: warp-specialised + persistent conv tiles — numerics tests, per-shape
# cold A/B against the v2 tiles, then (TUNE=1) tuning-table adoption + interleaved bench
# A/B (tools/gpu_ws_tune.sh). Each GPU step has its own time limit; a crash ends the call.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_ws_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ws_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/ws_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/conv_ws_ab.py --out gpurun_out/ws_ab.json > gpurun_out/ws_ab.log 2>&1 || { tail -20 gpurun_out/ws_ab.log; exit 1; }
grep -v "^    " gpurun_out/ws_ab.log | grep -v amdgpu.ids
if [ -n "$TUNE" ]; then
  bash tools/gpu_ws_tune.sh
fi
