#!/bin/bash
# Service depth sweep at world 1 (tools/serve_bench.py: outputs PUT into the store), then
# the full default bench.py line.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for d in ${DEPTHS:-4 8 16}; do
  timeout -k 10 300 python -u tools/serve_bench.py --resnet-images 51200 --inception-images 25600 --depth $d \
    > gpurun_out/svc_depth_$d.log 2>&1 || { tail -20 gpurun_out/svc_depth_$d.log; exit 1; }
  echo "depth $d: $(grep '"metric"' gpurun_out/svc_depth_$d.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["p50_latency_ms"], r["steps"])')"
done
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
grep '"metric"' gpurun_out/bench_full.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); s=r["service"]; print("bench", r["value"], r["models"]["InceptionV3"]["value"], "service", s["value"], s["vs_time_weighted_single_model"], s["p50_latency_ms"])'
