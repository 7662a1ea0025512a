#!/bin/bash
# PMC counters for a few conv shapes (counters-only runs: --pmc + --kernel-trace, nothing else).
#   ONLY=<layer substrings> CFGS=<cfg ids> tools/pmc_conv.sh
# Pass 1: wave-state / MFMA / LDS counters; pass 2: L2 (TCC) traffic. LIST=1 also
# dumps the available counter names.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
ONLY=${ONLY:-conv4_block1_2,conv2_block1_3,conv3_block1_2}
CFGS=${CFGS:-11,14,15}
if [ -n "$LIST" ]; then
  timeout -k 10 120 rocprofv3 --list-avail > $R/gpurun_out/pmc_avail.txt 2>&1 || true
fi
timeout -k 10 300 rocprofv3 --pmc ${PMC:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE} --kernel-trace --output-format csv -d $R/gpurun_out/pmc -o conv -- python3 $R/tools/conv_bench.py --only $ONLY --cfgs $CFGS --iters 2 > $R/gpurun_out/pmc.log 2>&1 && echo pmc-ok || { tail -20 $R/gpurun_out/pmc.log; exit 1; }
if [ -n "$L2" ]; then
  timeout -k 10 300 rocprofv3 --pmc ${L2_COUNTERS:-TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum} --kernel-trace --output-format csv -d $R/gpurun_out/pmc_l2 -o conv -- python3 $R/tools/conv_bench.py --only $ONLY --cfgs $CFGS --iters 2 > $R/gpurun_out/pmc_l2.log 2>&1 && echo pmc-l2-ok || { tail -20 $R/gpurun_out/pmc_l2.log; exit 1; }
fi
