#!/bin/bash
# One gpurun call for the generic row-ring family: its GPU numerics tests, then the per-layer cold
# A/B against the current tiles (tools/conv_ws_ab.py; SHAPES= narrows it), then optionally the
# tuning-table A/B (TABLES=...).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_rrg_gpu.py tests/test_conv_rr_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rrg_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/rrg_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/conv_ws_ab.py --shapes ${SHAPES:-inc_c5,inc_35_64_96,inc_35_96_96,inc_35_5x5,inc_17_1x7,inc_17_7x1,inc_17_7x1_192,inc_8_1x3,r50_3x3_s2,r50_3x3_s3,r50_3x3_s4} --v2 ${V2:-11,12,14,15,24,26,28,30,32} --ws ${WS:-102,104,121,122,125,127,150,$(seq -s, 160 177)} --out gpurun_out/rrg_ab.json > gpurun_out/rrg_ab.log 2>&1 || { tail -20 gpurun_out/rrg_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rrg_ab.log
if [ -n "$TABLES" ]; then
  bash tools/gpu_table_ab.sh || exit 1
fi
