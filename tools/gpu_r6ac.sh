#!/bin/bash
# r6 call AC: segments per image (256 / 512 / 128) with the single-path symbol decode, window bench x2.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_ac
mkdir -p $O
export TMPDIR=/tmp
DML_JPEG_PT=512 timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest512.log 2>&1 || { tail -20 $O/pytest512.log; exit 1; }
tail -1 $O/pytest512.log
for r in 1 2; do
  for v in 256 512 128; do
    DML_JPEG_PT=$v timeout -k 10 120 python tools/jpeg_bench.py > $O/bench_pt${v}_r$r.log 2>&1 || { tail -5 $O/bench_pt${v}_r$r.log; exit 1; }
    echo "PT=$v r$r: $(grep -h window $O/bench_pt${v}_r$r.log | tr '\n' ' ')"
  done
done
