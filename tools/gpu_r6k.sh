#!/bin/bash
# r6 call K: the parallel Huffman kernel with its entropy stream staged in LDS (DML_JPEG_LDS=1,
# default) against global-memory reads (=0): JPEG numerics, the window bench interleaved, one
# kernel-trace pass each, then the 51,200-distinct service pass both ways.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6_lds
export TMPDIR=/tmp
O=gpurun_out/r6_lds
timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py tests/test_jpeg_decode.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 1 0; do
    DML_JPEG_LDS=$v timeout -k 10 120 python tools/jpeg_bench.py > $O/bench_lds${v}_r$r.log 2>&1 || { tail -5 $O/bench_lds${v}_r$r.log; exit 1; }
    echo "LDS=$v r$r: $(grep -h window $O/bench_lds${v}_r$r.log | tr '\n' ' ')"
  done
done
for v in 1 0; do
  DML_JPEG_LDS=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_lds$v -o run -- python3 tools/jpeg_bench.py > $O/prof_lds$v.log 2>&1 || { tail -5 $O/prof_lds$v.log; exit 1; }
done
find $O -name '*kernel_stats.csv' | sort | while read f; do echo "$f"; grep -h jpeg "$f" | cut -d, -f1-4; done
for v in 1 0; do
  DML_JPEG_LDS=$v timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/distinct_lds$v.log 2>&1 || { tail -20 $O/distinct_lds$v.log; exit 1; }
  echo "LDS=$v"; python tools/bench_summary.py $O/distinct_lds$v.log
done
