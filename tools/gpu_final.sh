#!/bin/bash
# Round-end measurements: headline bench (both models), the single-engine
# (--splits 1) variant, and a longer concurrent service run. Own limit per step.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-200 || { tail -30 gpurun_out/bench.log; exit 1; }
timeout -k 10 600 python bench.py --steps 30 --warmup 5 --splits 1 > gpurun_out/bench_splits1.log 2>&1 && tail -1 gpurun_out/bench_splits1.log | cut -c1-200 || { tail -30 gpurun_out/bench_splits1.log; exit 1; }
timeout -k 10 600 python tools/serve_bench.py --resnet-images 102400 --inception-images 51200 > gpurun_out/serve_bench.log 2>&1 && tail -1 gpurun_out/serve_bench.log | cut -c1-300 || { tail -30 gpurun_out/serve_bench.log; exit 1; }
