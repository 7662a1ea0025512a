#!/bin/bash
# Full GPU suite, then InceptionV3 b128 sub-batch layouts re-checked with the grouped launches.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
i=0
for v in "--splits 2" "--splits 1" "--splits 4 --streams 2" "--splits 4" "--splits 2 --lookahead 2"; do
  i=$((i+1))
  timeout -k 10 600 python bench.py --model InceptionV3 --steps 30 --warmup 5 $v > gpurun_out/inc_split$i.log 2>&1 \
    && echo "$v: $(tail -1 gpurun_out/inc_split$i.log | cut -c1-120)" || { tail -20 gpurun_out/inc_split$i.log; exit 1; }
done
