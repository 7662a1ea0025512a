#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python tools/conv_bench.py --model InceptionV3 --batch 128 --out gpurun_out/conv_bench_inc.json > gpurun_out/conv_bench_inc.log 2>&1 && tail -2 gpurun_out/conv_bench_inc.log && \
timeout -k 10 600 python bench.py --model InceptionV3 --steps 20 --warmup 5 --op-times gpurun_out/op_times_inc.json > gpurun_out/bench_inc.log 2>&1 && tail -1 gpurun_out/bench_inc.log
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/ 2>/dev/null || true
