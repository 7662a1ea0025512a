#!/bin/bash
# One gpurun call: the store path on the GPU — the resize kernel test, the serving GPU tests
# (store windows, jobs larger than the arena), then the default bench (headline + service +
# store-image pass) with the GPU resize and (A/B) with the Pillow resize in the decode pool.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_resize_gpu.py tests/test_serving_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/store_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/store_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
python tools/bench_summary.py gpurun_out/bench_full.log
DML_GPU_RESIZE=0 timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_cpuresize.log 2>&1 || { tail -30 gpurun_out/bench_cpuresize.log; exit 1; }
python tools/bench_summary.py gpurun_out/bench_cpuresize.log
