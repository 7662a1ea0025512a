#!/bin/bash
# One gpurun call for new conv tiles: numerics tests of the ws / wsp / pt tiles, the per-shape
# cold A/B against the v2 tiles (tools/conv_ws_ab.py; SHAPES= / WS= narrow it), then (TUNE=1)
# tuning-table adoption of ADD=<ids> with an interleaved bench A/B (tools/gpu_ws_tune.sh).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_conv_rr_gpu.py tests/test_conv_ws_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/conv_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/conv_ws_ab.py ${SHAPES:+--shapes $SHAPES} ${WS:+--ws $WS} --out gpurun_out/conv_ab.json > gpurun_out/conv_ab.log 2>&1 || { tail -20 gpurun_out/conv_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/conv_ab.log | grep -v "^    "
if [ -n "$TUNE" ]; then
  bash tools/gpu_ws_tune.sh || exit 1
fi
