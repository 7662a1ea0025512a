#!/bin/bash
# scratch gpurun command for the current A/B (overwritten per experiment)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_bneck.log 2>&1 && tail -3 gpurun_out/pt_bneck.log &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b_fused.log 2>&1 && tail -1 gpurun_out/b_fused.log | cut -c1-200 &&
DML_FUSED_BLOCKS=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b_unfused.log 2>&1 && tail -1 gpurun_out/b_unfused.log | cut -c1-200
