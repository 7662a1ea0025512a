#!/bin/bash
# Final r4 evidence: default bench line (both models + service), service kernel census, bench kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/final_bench.log 2>&1 || { tail -30 gpurun_out/final_bench.log; exit 1; }
grep '"metric"' gpurun_out/final_bench.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); s=r["service"]; print("bench", r["value"], r["models"]["InceptionV3"]["value"], "service", s["value"], s["vs_time_weighted_single_model"], s["p50_latency_ms"])'
RI=25600 II=12800 bash tools/gpu_svc_prof.sh > gpurun_out/final_census.out 2>&1 || { tail -20 gpurun_out/final_census.out; exit 1; }
tail -12 gpurun_out/final_census.out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o bench -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-service > $R/gpurun_out/prof_bench.log 2>&1 || { tail -20 $R/gpurun_out/prof_bench.log; exit 1; }
python3 $R/tools/kernel_census.py $R/gpurun_out/prof_bench | head -30
