#!/bin/bash
# r6 call E: GPU JPEG numerics after the batched native slot / re-target calls, then the
# 51,200-distinct pass twice (plain, then with the serve loop under cProfile).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py tests/test_rank_service_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/e_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/e_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-service > gpurun_out/e_bench.log 2>&1 || { tail -20 gpurun_out/e_bench.log; exit 1; }
python tools/bench_summary.py gpurun_out/e_bench.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > gpurun_out/distinct_e.log 2>&1 || { tail -20 gpurun_out/distinct_e.log; exit 1; }
python tools/bench_summary.py gpurun_out/distinct_e.log
grep -o '"decode_pool_s_coordinator": {[^}]*}' gpurun_out/distinct_e.log || true
grep -o '"loop_phase_s": {[^}]*}' gpurun_out/distinct_e.log | tail -1 || true
DML_PROFILE_SERVE=$PWD/gpurun_out/serve_profile.txt timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > gpurun_out/distinct_e_prof.log 2>&1 || { tail -20 gpurun_out/distinct_e_prof.log; exit 1; }
python tools/bench_summary.py gpurun_out/distinct_e_prof.log
head -60 gpurun_out/serve_profile.txt
