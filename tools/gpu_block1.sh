set -o pipefail
cd $GRAFT_REPO_ROOT
export DML_SKIP_BUILD=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_block_fused_gpu.py > gpurun_out/g2_test.log 2>&1 && \
timeout -k 10 300 python -u tools/block_bench.py --out gpurun_out/g2_bench.json > gpurun_out/g2_bench.log 2>&1
