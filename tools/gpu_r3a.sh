# round-3 validation: engine numerics (new calibrated oracle), serving on GPU, fused block, smoke, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export DML_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_serving_gpu.py tests/test_block_fused_gpu.py > gpurun_out/r3a_pytest.log 2>&1 && \
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/r3a_smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r3a_bench.log 2>&1
