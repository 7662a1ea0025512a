timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py -k "pool_gemm" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_pg.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_pg.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="-;DML_CHAIN_MERGED=1" ROUNDS=3 BENCH_ARGS="--models ResNet50 --no-service" bash tools/gpu_env_ab.sh && mkdir -p gpurun_out/r50 && mv gpurun_out/envab_* gpurun_out/r50/ &&
VARIANTS="-;DML_POOL_GEMM=1" ROUNDS=3 BENCH_ARGS="--models InceptionV3 --no-service" bash tools/gpu_env_ab.sh &&
DML_POOL_GEMM=1 timeout -k 10 300 python tools/op_times.py --runs InceptionV3:64 --out-dir gpurun_out/ops_pg && python -c "
import json; d=json.load(open('gpurun_out/ops_pg/op_times_InceptionV3_b64.json'))
print([(n, round(t*1000,1)) for n,t in d['ops'][:6]])"
