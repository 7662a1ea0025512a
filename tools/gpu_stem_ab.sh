#!/bin/bash
# Stem iteration: stem GPU tests, stem microbench, then interleaved ResNet50 bench rounds with the
# folded stem 1x1 on (default) and off (DML_FOLD_STEM_1X1=0).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 240 \
  --timeout-method thread > gpurun_out/stem_tests.log 2>&1; rc=$?
tail -2 gpurun_out/stem_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/stem_bench.py --out gpurun_out/stem_bench3.json > gpurun_out/stem_bench3.log 2>&1 \
  && grep -v amdgpu.ids gpurun_out/stem_bench3.log || exit 1
for r in 1 2; do
  for f in 1 0; do
    DML_FOLD_STEM_1X1=$f timeout -k 10 300 python -u bench.py --model ResNet50 --steps 30 --warmup 5 --no-service \
      > gpurun_out/fold_${f}_$r.log 2>&1 || { tail -20 gpurun_out/fold_${f}_$r.log; exit 1; }
    echo "fold $f round $r: $(grep '"metric"' gpurun_out/fold_${f}_$r.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  done
done
