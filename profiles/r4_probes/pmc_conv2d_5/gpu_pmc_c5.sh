#!/bin/bash
# InceptionV3 conv2d_5 (3x3 80 -> 192, b64) on tiles 15 (2-stage) and 38 (3-stage): counter
# passes, each its own run (--pmc + --kernel-trace only). PASS=list|sq|ta|td
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/tools/conv_bench.py --model InceptionV3 --batch 64 --only conv2d_5 --cfgs 15,38 --iters 3"
for p in ${PASSES:-list sq}; do
  case $p in
    list) timeout -k 10 120 rocprofv3 --list-avail > $R/gpurun_out/pmc_avail.txt 2>&1; echo list-rc $? ;;
    sq) timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_c5_sq -o c5 -- $CMD > $R/gpurun_out/pmc_c5_sq.log 2>&1 && echo sq-ok || { tail -5 $R/gpurun_out/pmc_c5_sq.log; exit 1; } ;;
    *) timeout -s KILL 120 rocprofv3 --pmc $(echo ${!p}) GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_c5_$p -o c5 -- $CMD > $R/gpurun_out/pmc_c5_$p.log 2>&1 && echo $p-ok || { tail -5 $R/gpurun_out/pmc_c5_$p.log; exit 1; } ;;
  esac
done
