#!/bin/bash
# r6 call R (final tree): the full GPU suite, the driver's bench command, then kernel traces of the
# driver's command and of the 51,200-distinct pass (stats + store-pass timeline).
set -o pipefail
cd "$(dirname "$0")/.."
O=$PWD/gpurun_out/r6_r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python tools/bench_summary.py $O/bench.log
R=$PWD
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_distinct -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 5 --warmup 2 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/prof_distinct.log 2>&1 || { tail -20 $O/prof_distinct.log; exit 1; }
cd $R && python tools/trace_store_pass.py $(find $O/prof_distinct -name '*kernel_trace.csv' | head -1) > $O/distinct_timeline.json && cat $O/distinct_timeline.json | head -30
find $O/prof_distinct -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $O/distinct_kernel_stats.csv
find $O/prof_distinct -name '*kernel_trace.csv' -delete
