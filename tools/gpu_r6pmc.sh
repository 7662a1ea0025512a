#!/bin/bash
# r6 PMC passes (one counter set per run, kernel trace only): the parallel Huffman kernel (JPEG
# window bench) and InceptionV3's ops (op_times, 64-image sub-batch).
set -o pipefail
cd "$(dirname "$0")/.."
O=$PWD/gpurun_out/r6_pmc
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" $O/avail.txt | sort -u > $O/sq_counters.txt || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d $O/huff -o run --output-format csv -- python3 $R/tools/jpeg_bench.py --iters 3 --windows 1 > $O/huff.log 2>&1 && echo huff-ok || echo huff-failed
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d $O/inc -o run --output-format csv -- python3 $R/tools/op_times.py --runs InceptionV3:64 --passes 1 --out-dir $O/ops > $O/inc.log 2>&1 && echo inc-ok || echo inc-failed
cd $R
find $O -name '*counter_collection.csv' | head -5
