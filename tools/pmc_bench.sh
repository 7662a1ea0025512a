#!/bin/bash
# One counters-only rocprofv3 pass (--pmc + --kernel-trace, nothing else) over a short ResNet50
# bench: wave-state / MFMA / LDS counters per dispatch -> gpurun_out/pmc_bench/ (summarise with
# tools/pmc_summary.py). Kernels are serialised by the collection.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_bench
cd /tmp && export TMPDIR=/tmp DML_SKIP_BUILD=1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $R/gpurun_out/pmc_bench/p1 -o run -- \
  python3 $R/bench.py --models ${MODEL:-ResNet50} --no-service --steps 2 --warmup 1 --no-verify > $R/gpurun_out/pmc_bench/p1.log 2>&1
