set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "softmax or split_k" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_sm.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_sm.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="-;DML_SOFTMAX_WG=1" ROUNDS=2 BENCH_ARGS="--models ResNet50 --no-service" bash tools/gpu_env_ab.sh && mkdir -p gpurun_out/r50 && mv gpurun_out/envab_* gpurun_out/r50/ &&
VARIANTS="-;DML_SOFTMAX_WG=1" ROUNDS=2 BENCH_ARGS="--models InceptionV3 --no-service" bash tools/gpu_env_ab.sh
