#!/bin/bash
# r6 call G: kernel trace of the 51,200-distinct store-image pass (model vs JPEG kernels).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_distinct -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 5 --warmup 2 --models ResNet50 --svc-store-images 51200 --kill-pass off > $GRAFT_REPO_ROOT/gpurun_out/prof_distinct.log 2>&1 && echo profiled || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_distinct.log; exit 1; }
cd $GRAFT_REPO_ROOT && python tools/bench_summary.py gpurun_out/prof_distinct.log
