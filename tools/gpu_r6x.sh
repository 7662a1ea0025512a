#!/bin/bash
# r6 call X: one-rank time slicing of the two jobs (config 4 at 1 GPU): the service GPU tests,
# then the driver's bench command twice (its service record shows the split and both rates).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_rank_service_gpu.py tests/test_serving_gpu.py -x -q --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_r$r.log 2>&1 || { tail -20 $O/bench_r$r.log; exit 1; }
  python tools/bench_summary.py $O/bench_r$r.log
  python - <<PY
import json
l = [x for x in open("$O/bench_r$r.log") if x.startswith('{"metric"')][-1]
s = json.loads(l)["service"]
print(" split", s.get("fair_share_splits"), "images/s", s.get("images_per_s"), "p50", s.get("p50_latency_ms"))
PY
done
