# round-3: chained-GEMM block boundary (C = 512): numerics, microbench vs two launches and the r1 kernel, pipeline A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export DML_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_stem_gpu.py -k "expand_reduce" > gpurun_out/r3f_test.log 2>&1 && \
timeout -k 10 300 python -u tools/chain_bench.py --out gpurun_out/r3f_chain.json > gpurun_out/r3f_chain.log 2>&1 && \
DML_CHAIN=0 timeout -k 10 300 python -u tools/chain_bench.py --out gpurun_out/r3f_chain_r1.json > gpurun_out/r3f_chain_r1.log 2>&1 && \
DML_CHAIN=1 timeout -k 10 300 python -u bench.py --models ResNet50 --no-service --steps 60 > gpurun_out/r3f_bench_chain.log 2>&1 && \
timeout -k 10 300 python -u bench.py --models ResNet50 --no-service --steps 60 > gpurun_out/r3f_bench_base.log 2>&1 && \
DML_CHAIN=1 timeout -k 10 300 python -u bench.py --models ResNet50 --no-service --steps 60 > gpurun_out/r3f_bench_chain2.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_stem_gpu.py -k "engine_fused" > gpurun_out/r3f_engine.log 2>&1
