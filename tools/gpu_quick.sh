#!/bin/bash
# One gpurun call for an iteration: selected GPU tests, then short benches of the
# listed models (service pass off), per-op times, the tuning table back.
#   TESTS="tests/test_kernels_gpu.py"  MODELS="ResNet50 InceptionV3"  STEPS=20  BENCH_ARGS=""
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1; rc=$?
  tail -15 gpurun_out/pytest_quick.log
  [ $rc -eq 0 ] || exit $rc
fi
for m in ${MODELS:-}; do
  timeout -k 10 600 python -u bench.py --model $m --steps ${STEPS:-20} --warmup 5 --no-service $BENCH_ARGS \
    --op-times gpurun_out/op_times_$m.json > gpurun_out/bench_$m.log 2>&1 && tail -1 gpurun_out/bench_$m.log | cut -c1-400 \
    || { tail -30 gpurun_out/bench_$m.log; exit 1; }
done
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/ 2>/dev/null || true
