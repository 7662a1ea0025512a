#!/bin/bash
# One gpurun call: the default bench (the driver's record: headline + service + store-image
# pass), the library-GEMM probe of the 1x1 shapes, and PMC counters of the 3x3 tiles
# (v2 11 / ws 102 / pt 140, 141) on two ResNet50 shapes. Each GPU step has its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out/pmc_pt
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
python tools/bench_summary.py gpurun_out/bench_full.log
timeout -k 10 600 python -u tools/conv_ws_ab.py --shapes r50_3x3_s2,r50_3x3_s3,r50_3x3_s4,r50_3x3_s5,inc_35_64_96,inc_8_448_384 --ws 102,119,126,127,140,141,144,147,148,149 --out gpurun_out/ws_ab_deep.json > gpurun_out/ws_ab_deep.log 2>&1 || { tail -20 gpurun_out/ws_ab_deep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ws_ab_deep.log
timeout -k 10 300 python -u tools/gemm_probe.py --out gpurun_out/gemm_probe.json > gpurun_out/gemm_probe.log 2>&1 || { tail -20 gpurun_out/gemm_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gemm_probe.log
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_pt -o p1 -- python3 $R/tools/conv_pmc_run.py --shapes r50_3x3_s4,r50_3x3_s3 --cfgs 11,102,119,140,147 --iters 3 > $R/gpurun_out/pmc_pt1.log 2>&1 && echo pmc1-ok || { tail -5 $R/gpurun_out/pmc_pt1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVES SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_pt -o p2 -- python3 $R/tools/conv_pmc_run.py --shapes r50_3x3_s4,r50_3x3_s3 --cfgs 11,102,119,140,147 --iters 3 > $R/gpurun_out/pmc_pt2.log 2>&1 && echo pmc2-ok || { tail -5 $R/gpurun_out/pmc_pt2.log; exit 1; }
