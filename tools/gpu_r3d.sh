# round-3: shifted-pixel stride-1 conv kernel: numerics, microbench; GPU launcher CLI test
set -o pipefail
cd $GRAFT_REPO_ROOT
export DML_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_shift_gpu.py > gpurun_out/r3d_test.log 2>&1 && \
timeout -k 10 400 python -u tools/shift_bench.py --out gpurun_out/r3d_shift.json > gpurun_out/r3d_shift.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_rank_service_gpu.py > gpurun_out/r3d_rank.log 2>&1
