#!/bin/bash
# New tile configs: kernel numerics, then a fresh tuning table (new candidate
# tag) built by the bench of both models, the InceptionV3 per-op times and the table.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/tiles
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  > gpurun_out/tiles/pytest.log 2>&1 || { tail -40 gpurun_out/tiles/pytest.log; exit 1; }
tail -2 gpurun_out/tiles/pytest.log
timeout -k 10 600 python bench.py --steps 30 --warmup 5 > gpurun_out/tiles/bench.log 2>&1 \
  && tail -1 gpurun_out/tiles/bench.log | cut -c1-400 || { tail -30 gpurun_out/tiles/bench.log; exit 1; }
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/tiles/conv_tuning.json
timeout -k 10 300 python tools/group_ops.py > gpurun_out/tiles/ops.log 2>&1 && tail -3 gpurun_out/tiles/ops.log \
  || { tail -30 gpurun_out/tiles/ops.log; exit 1; }
cp gpurun_out/groups/ops.json gpurun_out/tiles/ops.json
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/tiles/conv_tuning.json
