#!/bin/bash
# r6 call AD (final tree): kernel trace of the 51,200-distinct pass (store-pass timeline) and of
# the driver's command (kernel stats).
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$PWD/gpurun_out/r6_ad
mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_distinct -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 5 --warmup 2 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/prof_distinct.log 2>&1) || { tail -20 $O/prof_distinct.log; exit 1; }
python tools/trace_store_pass.py $(find $O/prof_distinct -name '*kernel_trace.csv' | head -1) > $O/distinct_timeline.json && head -24 $O/distinct_timeline.json
find $O/prof_distinct -name '*kernel_trace.csv' -delete
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_driver -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-service > $O/prof_driver.log 2>&1) || { tail -20 $O/prof_driver.log; exit 1; }
find $O/prof_driver -name '*kernel_trace.csv' -delete
python tools/bench_summary.py $O/prof_driver.log
