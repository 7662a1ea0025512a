#!/bin/bash
# PMC counters for a few conv shapes (counters-only run: --pmc + --kernel-trace, nothing else).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc -o conv -- python3 $R/tools/conv_bench.py --only ${ONLY:-conv4_block1_2,conv2_block1_3,conv3_block1_2} --cfgs ${CFGS:-11,14,15} --iters 2 > $R/gpurun_out/pmc.log 2>&1 && echo pmc-ok || { tail -20 $R/gpurun_out/pmc.log; exit 1; }
