#!/bin/bash
# PMC counters of the fused stem / conv+pool kernels (counters-only pass:
# --pmc + --kernel-trace, nothing else), plus their plain timings.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/fused_kernels_probe.py > $R/gpurun_out/fused_times.log 2>&1 && cat $R/gpurun_out/fused_times.log | grep us || exit 1
timeout -k 10 -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fused -o fused -- python3 $R/tools/fused_kernels_probe.py --iters 2 > $R/gpurun_out/pmc_fused.log 2>&1 && echo pmc-ok || { tail -20 $R/gpurun_out/pmc_fused.log; exit 1; }
