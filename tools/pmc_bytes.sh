#!/bin/bash
# HBM bytes per conv dispatch: FETCH_SIZE and WRITE_SIZE (KB) in two counter-only
# passes (rocprofv3 --pmc + --kernel-trace, nothing else), plus the practical
# HBM ceilings of this box (tools/hbm_bw.py).
#   ONLY=<layer substrings> CFGS=<cfg ids> BATCH=128 tools/pmc_bytes.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
ONLY=${ONLY:-conv2_block2_3,conv2_block2_1,conv3_block2_3,conv3_block2_1,conv4_block2_3}
CFGS=${CFGS:-14}
BATCH=${BATCH:-128}
timeout -k 10 120 python3 $R/tools/hbm_bw.py $R/gpurun_out/hbm_bw.json > $R/gpurun_out/hbm_bw.log 2>&1 && tail -1 $R/gpurun_out/hbm_bw.log || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc_$C -o conv -- python3 $R/tools/conv_bench.py --batch $BATCH --only $ONLY --cfgs $CFGS --iters 2 > $R/gpurun_out/pmc_$C.log 2>&1 && echo "pmc $C ok" || { tail -20 $R/gpurun_out/pmc_$C.log; exit 1; }
done
