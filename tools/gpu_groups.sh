#!/bin/bash
# Grouped InceptionV3 branch convs: kernel + engine numerics, then the bench
# (InceptionV3 only) with and without grouping, then per-op times of both plans.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/groups
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "group or oracle" > gpurun_out/groups/pytest.log 2>&1 \
  || { tail -40 gpurun_out/groups/pytest.log; exit 1; }
tail -2 gpurun_out/groups/pytest.log
grep "grouped launches" gpurun_out/groups/pytest.log || true
for G in 1 0; do
  DML_CONV_GROUPS=$G timeout -k 10 400 python bench.py --steps 30 --warmup 5 --models InceptionV3 \
    > gpurun_out/groups/bench_g$G.log 2>&1 && tail -1 gpurun_out/groups/bench_g$G.log \
    || { tail -30 gpurun_out/groups/bench_g$G.log; exit 1; }
done
timeout -k 10 300 python tools/group_ops.py > gpurun_out/groups/ops.log 2>&1 && tail -25 gpurun_out/groups/ops.log \
  || { tail -30 gpurun_out/groups/ops.log; exit 1; }
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/groups/conv_tuning.json
