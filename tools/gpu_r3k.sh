# round-3: chained block boundaries - big-step variant, merged stage entries (C = 256 / 512), C = 256
# boundary: numerics, microbench, pipeline A/B (interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
export DML_SKIP_BUILD=1
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_stem_gpu.py"
timeout -k 10 300 $T -k "expand_reduce" > gpurun_out/r3k_test.log 2>&1 && \
DML_CHAIN_BIG=1 timeout -k 10 300 $T -k "chain" > gpurun_out/r3k_test_big.log 2>&1 && \
DML_CHAIN_C256=1 timeout -k 10 300 $T -k "expand_reduce_matches or subsampled" > gpurun_out/r3k_test_c256.log 2>&1 && \
DML_CHAIN_MERGED=1 timeout -k 10 300 $T -k "engine_fused" > gpurun_out/r3k_test_engine_merged.log 2>&1 && \
DML_CHAIN_BIG=1 timeout -k 10 300 python -u tools/chain_bench.py --out gpurun_out/r3k_chain_big.json > gpurun_out/r3k_chain_big.log 2>&1 && \
DML_CHAIN_BIG=1 timeout -k 10 300 python -u tools/chain_bench.py --c 1024 --out gpurun_out/r3k_chain_big1024.json > gpurun_out/r3k_chain_big1024.log 2>&1 && \
B="python -u bench.py --models ResNet50 --no-service --steps 100" && \
timeout -k 10 300 $B > gpurun_out/r3k_base_a.log 2>&1 && \
DML_CHAIN_BIG=1 timeout -k 10 300 $B > gpurun_out/r3k_big_a.log 2>&1 && \
DML_CHAIN_MERGED=1 timeout -k 10 300 $B > gpurun_out/r3k_merged_a.log 2>&1 && \
DML_CHAIN_MERGED=1 DML_CHAIN_C256=1 timeout -k 10 300 $B > gpurun_out/r3k_mc256_a.log 2>&1 && \
timeout -k 10 300 $B > gpurun_out/r3k_base_b.log 2>&1 && \
DML_CHAIN_BIG=1 timeout -k 10 300 $B > gpurun_out/r3k_big_b.log 2>&1 && \
DML_CHAIN_MERGED=1 timeout -k 10 300 $B > gpurun_out/r3k_merged_b.log 2>&1 && \
DML_CHAIN_MERGED=1 DML_CHAIN_C256=1 timeout -k 10 300 $B > gpurun_out/r3k_mc256_b.log 2>&1 &&
timeout -k 10 300 $T -k "folded or folds" > gpurun_out/r3k_test_fold.log 2>&1 && \
BI="python -u bench.py --models InceptionV3 --no-service --steps 100" && \
timeout -k 10 300 $BI > gpurun_out/r3k_inc_fold_a.log 2>&1 && \
DML_FOLD_POOL_1X1=0 timeout -k 10 300 $BI > gpurun_out/r3k_inc_nofold_a.log 2>&1 && \
timeout -k 10 300 $BI > gpurun_out/r3k_inc_fold_b.log 2>&1 && \
DML_FOLD_POOL_1X1=0 timeout -k 10 300 $BI > gpurun_out/r3k_inc_nofold_b.log 2>&1
