#!/bin/bash
# One gpurun call: GPU tests, short benches (both models), optional variants and a
# rocprofv3 kernel-stats profile. Every GPU step has its own time limit; steps are
# chained so the first failure (fault, abort, timeout) ends the call.
#   PROFILE=1  add a rocprofv3 --kernel-trace --stats run of the ResNet50 bench
#   VARIANTS="--splits 4 --streams 2;--splits 1"  extra ResNet50 bench lines
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-20}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -15 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || [ -n "$CONTINUE_ON_TEST_FAIL" ] || exit $rc
fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 --op-times gpurun_out/op_times.json > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log || { tail -30 gpurun_out/bench.log; exit 1; }
timeout -k 10 600 python bench.py --model InceptionV3 --steps $STEPS --warmup 5 --op-times gpurun_out/op_times_inc.json > gpurun_out/bench_inc.log 2>&1 && tail -1 gpurun_out/bench_inc.log || { tail -30 gpurun_out/bench_inc.log; exit 1; }
i=0
IFS=';' read -ra VS <<< "${VARIANTS:-}"
for v in "${VS[@]}"; do
  i=$((i+1))
  timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 $v > gpurun_out/bench_var$i.log 2>&1 && echo "variant $i ($v): $(tail -1 gpurun_out/bench_var$i.log | cut -c1-140)" || { tail -30 gpurun_out/bench_var$i.log; exit 1; }
done
if [ -n "$PROFILE" ]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 && echo profiled || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit 1; }
fi
cp $GRAFT_REPO_ROOT/distributed_machine_learning_amd/tuning/conv_tuning.json $GRAFT_REPO_ROOT/gpurun_out/ 2>/dev/null || true
