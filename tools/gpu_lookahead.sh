#!/bin/bash
# Dispatch lookahead 2 vs 1: throughput and p50/p90 query latency (both models),
# plus the pipeline GPU tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/la
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_serving_gpu.py -k pipeline \
  > gpurun_out/la/pytest.log 2>&1 || { tail -30 gpurun_out/la/pytest.log; exit 1; }
tail -1 gpurun_out/la/pytest.log
for la in 2 1 2 1; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --lookahead $la > gpurun_out/la/b$la.log 2>&1 || { tail -20 gpurun_out/la/b$la.log; exit 1; }
  python - "$la" <<'PY'
import json, sys
la = sys.argv[1]
d = json.loads(open(f"gpurun_out/la/b{la}.log").read().strip().splitlines()[-1])
i = d["models"]["InceptionV3"]
print(f"lookahead {la}: ResNet50 {d['value']:.0f} img/s p50 {d['p50_latency_ms']} p90 {d['p90_latency_ms']} | "
      f"InceptionV3 {i['value']:.0f} p50 {i['p50_latency_ms']} p90 {i['p90_latency_ms']}")
PY
done
