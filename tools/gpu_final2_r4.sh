#!/bin/bash
# Round-end rehearsal on the final tree: full GPU suite, smoke, default bench line.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
NO_AB=1 bash tools/gpu_full_r4.sh || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/final2_bench.log 2>&1 || { tail -30 gpurun_out/final2_bench.log; exit 1; }
grep '"metric"' gpurun_out/final2_bench.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); s=r["service"]; print("bench", r["value"], r["models"]["InceptionV3"]["value"], "service", s["value"], s["vs_time_weighted_single_model"], s["p50_latency_ms"])'
