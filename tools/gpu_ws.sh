#!/bin/bash
# conv_ws.hip (persistent weight-stationary 1x1) vs the v2 tiles, per 1x1 shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ws_bench.py --iters 20 --clean-scrub --out gpurun_out/ws_bench_clean.json > gpurun_out/ws_bench_clean.log 2>&1
rc=$?
cat gpurun_out/ws_bench_clean.log
exit $rc
