#!/bin/bash
# PMC counter passes (counters only: --pmc + --kernel-trace, nothing else) over the chained
# block-boundary kernel (tools/chain_bench.py) and one implicit-GEMM conv (tools/conv_one.py).
# Pass 1: wave state / MFMA / LDS; pass 2: L2 (TCC) traffic. Each pass its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_r3
cd /tmp && export TMPDIR=/tmp DML_SKIP_BUILD=1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $R/gpurun_out/pmc_r3/chain_p1 -o run -- python3 $R/tools/chain_bench.py --iters 3 > $R/gpurun_out/pmc_r3/chain_p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d $R/gpurun_out/pmc_r3/chain_p2 -o run -- python3 $R/tools/chain_bench.py --iters 3 > $R/gpurun_out/pmc_r3/chain_p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $R/gpurun_out/pmc_r3/conv_s4_p1 -o run -- python3 $R/tools/conv_one.py --shape r50_s4_3x3 --cfg 11 --iters 20 > $R/gpurun_out/pmc_r3/conv_p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $R/gpurun_out/pmc_r3/shift_s4_p1 -o run -- python3 $R/tools/conv_one.py --shape r50_s4_3x3 --cfg 64 --iters 20 > $R/gpurun_out/pmc_r3/shift_p1.log 2>&1
