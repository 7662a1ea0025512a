#!/bin/bash
# Stem kernels: numerics, then per-op times of both models and the bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/stem
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_stem_gpu.py \
  tests/test_engine_gpu.py -k "stem or oracle" > gpurun_out/stem/pytest.log 2>&1 || { tail -40 gpurun_out/stem/pytest.log; exit 1; }
tail -1 gpurun_out/stem/pytest.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --op-times gpurun_out/stem/op_times.json > gpurun_out/stem/bench.log 2>&1 \
  || { tail -30 gpurun_out/stem/bench.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/stem/bench.log").read().strip().splitlines()[-1])
print("bench ResNet50", d["value"], "InceptionV3", d["models"]["InceptionV3"]["value"])
for f in ("gpurun_out/stem/op_times.json", "gpurun_out/stem/op_times_InceptionV3.json"):
    o = json.load(open(f))
    for n, t in o["ops"]:
        if "preprocess" in n or "+max_pooling2d_1" in n:
            print(o["model"], n, round(t * 1e3, 1), "us")
    print(o["model"], "total", round(o["total_ms"], 3), "ms")
PY
