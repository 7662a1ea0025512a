#!/bin/bash
# Winograd kernel A/B: tools/wino_bench.py over the listed variant libraries, optionally a
# counters-only rocprofv3 pass over the cfg-80 launches (PMC=1).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/wino_bench.py --cfgs ${CFGS:-80,11,15,30,32,12,14} --lib "${LIBS:-}" \
  --out gpurun_out/wino_bench.json > gpurun_out/wino_bench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/wino_bench.log | tail -20
[ $rc -eq 0 ] || exit $rc
if [ -n "$PMC" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_wino -o wino -- python3 $R/tools/wino_bench.py --cfgs 80,11 --iters 2 > $R/gpurun_out/pmc_wino.log 2>&1 && echo pmc-ok || { tail -20 $R/gpurun_out/pmc_wino.log; exit 1; }
fi
