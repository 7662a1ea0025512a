# round-3: chained stage-3 boundary, big-step variant (one barrier per GEMM of a chunk): numerics, microbench, pipeline A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export DML_SKIP_BUILD=1
mkdir -p gpurun_out
DML_CHAIN_BIG=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem_gpu.py -k "chain" > gpurun_out/r3j_test.log 2>&1 && \
DML_CHAIN_BIG=1 timeout -k 10 300 python -u tools/chain_bench.py --out gpurun_out/r3j_chain_big.json > gpurun_out/r3j_chain_big.log 2>&1 && \
timeout -k 10 300 python -u tools/chain_bench.py --out gpurun_out/r3j_chain_4w.json > gpurun_out/r3j_chain_4w.log 2>&1 && \
B="python -u bench.py --models ResNet50 --no-service --steps 100" && \
timeout -k 10 300 $B > gpurun_out/r3j_4w_a.log 2>&1 && \
DML_CHAIN_BIG=1 timeout -k 10 300 $B > gpurun_out/r3j_big_a.log 2>&1 && \
timeout -k 10 300 $B > gpurun_out/r3j_4w_b.log 2>&1 && \
DML_CHAIN_BIG=1 timeout -k 10 300 $B > gpurun_out/r3j_big_b.log 2>&1
