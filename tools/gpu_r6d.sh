#!/bin/bash
# r6 call D: the whole GPU suite and smoke() (the driver's round-end checks), then a stage-depth
# A/B of the 51,200-distinct store-image pass.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log | cut -c1-200 || { tail -20 gpurun_out/smoke.log; exit 1; }
for d in 16 32; do
  DML_STAGE_DEPTH=$d timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > gpurun_out/distinct_sd$d.log 2>&1 || { tail -20 gpurun_out/distinct_sd$d.log; exit 1; }
  echo "stage depth $d: $(python tools/bench_summary.py gpurun_out/distinct_sd$d.log)"
done
