#!/bin/bash
# r6: parallel Huffman kernel after packing the table ids out of the symbol loop: numerics,
# the window bench twice, one PMC pass.
set -o pipefail
cd "$(dirname "$0")/.."
O=$PWD/gpurun_out/r6_pmc2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 120 python tools/jpeg_bench.py > $O/bench_r$r.log 2>&1 || { tail -5 $O/bench_r$r.log; exit 1; }
  grep -h window $O/bench_r$r.log | tr '\n' ' '; echo
done
R=$PWD
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d $O/huff -o run --output-format csv -- python3 $R/tools/jpeg_bench.py --iters 3 --windows 1 > $O/huff.log 2>&1 && echo huff-ok
