# round-3: persistent warp-specialised fused block: numerics (both kernels), microbench, pipeline A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export DML_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_block_fused_gpu.py > gpurun_out/r3c_test.log 2>&1 && \
timeout -k 10 300 python -u tools/block_bench.py --out gpurun_out/r3c_block.json > gpurun_out/r3c_block.log 2>&1 && \
DML_BLOCK_FUSED=1 timeout -k 10 300 python -u bench.py --models ResNet50 --no-service --steps 60 > gpurun_out/r3c_bench_blk.log 2>&1 && \
timeout -k 10 300 python -u bench.py --models ResNet50 --no-service --steps 60 > gpurun_out/r3c_bench_noblk.log 2>&1 && \
DML_BLOCK_FUSED=1 timeout -k 10 300 python -u bench.py --models ResNet50 --no-service --steps 60 > gpurun_out/r3c_bench_blk2.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_serving_gpu.py -k small_arena > gpurun_out/r3c_arena.log 2>&1
