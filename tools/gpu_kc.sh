#!/bin/bash
# After a kernel codegen change: kernel numerics, per-op times of both models, bench, service.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/kc
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  > gpurun_out/kc/pytest.log 2>&1 || { tail -30 gpurun_out/kc/pytest.log; exit 1; }
tail -1 gpurun_out/kc/pytest.log
timeout -k 10 200 python tools/op_times.py --out-dir gpurun_out/kc || exit 1
bash tools/gpu_sb_ab.sh
