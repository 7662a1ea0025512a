#!/bin/bash
# r6 call AA (re-run after the merged code / extra-bit shift): the single-path 11-bit Huffman symbol decode: numerics (Pillow byte-exact), the
# window bench twice, one PMC pass, then the 51,200-distinct pass twice.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$PWD/gpurun_out/r6_aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 120 python tools/jpeg_bench.py > $O/bench_r$r.log 2>&1 || { tail -5 $O/bench_r$r.log; exit 1; }
  grep -h window $O/bench_r$r.log | tr '\n' ' '; echo
done
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d $O/huff -o run --output-format csv -- python3 $R/tools/jpeg_bench.py --iters 3 --windows 1 > $O/huff.log 2>&1) && echo huff-ok
for r in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/distinct_r$r.log 2>&1 || { tail -20 $O/distinct_r$r.log; exit 1; }
  python tools/bench_summary.py $O/distinct_r$r.log
done
