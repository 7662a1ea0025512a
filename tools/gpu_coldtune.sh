#!/bin/bash
# Tuning-table A/B on one box: OLD tag table vs a NEW tag tuned in this call
# (cold-cache timing unless DML_TUNE_COLD=0), each bench run twice, interleaved.
#   OLD=c5cold NEW=c6cold [TESTS=1] tools/gpu_coldtune.sh
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
OLD=${OLD:-c5rt}; NEW=${NEW:-c5cold}
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
    -k "test_conv_matches_fp32 or test_conv_subsampled_residual" > gpurun_out/pytest_ct.log 2>&1; rc=$?
  tail -2 gpurun_out/pytest_ct.log; [ $rc -eq 0 ] || exit $rc
fi
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 900 python bench.py --steps 30 --warmup 5 > gpurun_out/ct_$n.log 2>&1 \
    && echo "$n: $(tail -1 gpurun_out/ct_$n.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["models"]["InceptionV3"]["value"], d["verified_top5"])')" \
    || { tail -20 gpurun_out/ct_$n.log; exit 1; }
}
run old1 DML_TUNING_TAG=$OLD $OLDENV
run tune DML_TUNING_TAG=$NEW
run new1 DML_TUNING_TAG=$NEW
run old2 DML_TUNING_TAG=$OLD $OLDENV
run new2 DML_TUNING_TAG=$NEW
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/conv_tuning_ct.json
