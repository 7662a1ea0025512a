# round-3 validation 2: numerics (RES_GAMMA 0.12), serving + rank launcher on GPU, smoke, default bench,
# then ResNet50 with the fused identity block (DML_BLOCK_FUSED=1) vs without, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
export DML_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py::test_engine_matches_oracle tests/test_serving_gpu.py tests/test_block_fused_gpu.py > gpurun_out/r3b_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/r3b_pytest.log
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/r3b_smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r3b_bench.log 2>&1 && \
DML_BLOCK_FUSED=1 timeout -k 10 300 python -u bench.py --models ResNet50 --no-service --steps 60 > gpurun_out/r3b_bench_blk.log 2>&1 && \
timeout -k 10 300 python -u bench.py --models ResNet50 --no-service --steps 60 > gpurun_out/r3b_bench_noblk.log 2>&1
