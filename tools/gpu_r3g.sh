# round-3: chained block boundary (C = 512 and 1024): numerics, 4- vs 8-wave workgroups, stamps, pipeline A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export DML_SKIP_BUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem_gpu.py -k "expand_reduce" > gpurun_out/r3g_test.log 2>&1 && \
DML_CHAIN_WAVES=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem_gpu.py -k "chain" > gpurun_out/r3g_test8.log 2>&1 && \
timeout -k 10 300 python -u tools/chain_bench.py --out gpurun_out/r3g_chain4.json > gpurun_out/r3g_chain4.log 2>&1 && \
DML_CHAIN_WAVES=8 timeout -k 10 300 python -u tools/chain_bench.py --out gpurun_out/r3g_chain8.json > gpurun_out/r3g_chain8.log 2>&1 && \
timeout -k 10 300 python -u tools/chain_bench.py --c 1024 --out gpurun_out/r3g_chain4_1024.json > gpurun_out/r3g_chain4_1024.log 2>&1 && \
DML_CHAIN_WAVES=8 timeout -k 10 300 python -u tools/chain_bench.py --c 1024 --out gpurun_out/r3g_chain8_1024.json > gpurun_out/r3g_chain8_1024.log 2>&1 && \
DML_CHAIN=1 timeout -k 10 300 python -u bench.py --models ResNet50 --no-service --steps 60 > gpurun_out/r3g_bench_chain4.log 2>&1 && \
timeout -k 10 300 python -u bench.py --models ResNet50 --no-service --steps 60 > gpurun_out/r3g_bench_base.log 2>&1 && \
DML_CHAIN=1 DML_CHAIN_WAVES=8 timeout -k 10 300 python -u bench.py --models ResNet50 --no-service --steps 60 > gpurun_out/r3g_bench_chain8.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_stem_gpu.py -k "engine_fused" > gpurun_out/r3g_engine.log 2>&1
