#!/bin/bash
# r6 call P: 512 vs 256 segments per image (numerics, window bench x2, 51,200-distinct pass).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_p
mkdir -p $O
export TMPDIR=/tmp
DML_JPEG_PT=512 timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest512.log 2>&1 || { tail -20 $O/pytest512.log; exit 1; }
tail -1 $O/pytest512.log
for r in 1 2; do
  for v in 256 512; do
    DML_JPEG_PT=$v timeout -k 10 120 python tools/jpeg_bench.py > $O/bench_pt${v}_r$r.log 2>&1 || { tail -5 $O/bench_pt${v}_r$r.log; exit 1; }
    echo "PT=$v r$r: $(grep -h window $O/bench_pt${v}_r$r.log | tr '\n' ' ')"
  done
done
for v in 512 256; do
  DML_JPEG_PT=$v timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/distinct_pt$v.log 2>&1 || { tail -20 $O/distinct_pt$v.log; exit 1; }
  echo "PT=$v $(python tools/bench_summary.py $O/distinct_pt$v.log)"
done
