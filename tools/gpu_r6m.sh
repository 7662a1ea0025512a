#!/bin/bash
# r6 call M: host JPEG prepare after the memchr un-stuffing / table cache, then the 51,200-distinct
# pass twice, then the world-8 capacity harness with the result collect on and off.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python tools/jpeg_bench.py > $O/jpeg_bench.log 2>&1 || { tail -5 $O/jpeg_bench.log; exit 1; }
cat $O/jpeg_bench.log | grep -v amdgpu.ids
for r in 1 2; do
  timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/distinct_r$r.log 2>&1 || { tail -20 $O/distinct_r$r.log; exit 1; }
  python tools/bench_summary.py $O/distinct_r$r.log
  grep -o '"decode_pool_s_coordinator": {[^}]*}' $O/distinct_r$r.log || true
done
for c in 1 0; do
  DML_COLLECT_RESULTS=$c timeout -k 10 240 python tools/store_capacity.py --world 8 --rate 600 --batches-per-rank 600 \
    --out $O/cap_c$c.json > $O/cap_c$c.log 2>&1 || { tail -20 $O/cap_c$c.log; exit 1; }
  echo "collect=$c $(grep -o '"batches_per_s": [0-9.]*' $O/cap_c$c.log | head -1)"
done
