#!/bin/bash
# Split-head / merged-tail A/B (SplitEngine(merge_at=...)): GPU tests of the mode, one untimed
# bench per merge point to tune the full-batch tail shapes (cached in the tuning table, copied
# to gpurun_out/), then interleaved rounds of the candidates.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_stem_gpu.py -k "split_engine or capture_parts or pool_gemm" -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_merge.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_merge.log
[ $rc -eq 0 ] || exit $rc
I1="InceptionV3=conv2d_31+conv2d_32+conv2d_35+conv2d_40"; I2="InceptionV3=conv2d_71+conv2d_73"
R1="ResNet50=conv4_block1_1_conv"; R2="ResNet50=conv5_block1_1_conv"
for m in "$I1" "$I2" "$R1" "$R2"; do
  model=${m%%=*}
  DML_MERGE_AT="$m" timeout -k 10 900 python bench.py --models $model --no-service --steps 10 --warmup 2 \
    > gpurun_out/tune_$model.log 2>&1 || { tail -20 gpurun_out/tune_$model.log; exit 1; }
  echo "tuned $m: $(tail -1 gpurun_out/tune_$model.log | grep -o '"value": [0-9.]*' | head -1)"
done
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/conv_tuning.json
VARIANTS="-;DML_POOL_GEMM=0;DML_MERGE_AT=$I1;DML_MERGE_AT=$I2" ROUNDS=2 BENCH_ARGS="--models InceptionV3 --no-service" \
  bash tools/gpu_env_ab.sh && mkdir -p gpurun_out/inc && mv gpurun_out/envab_* gpurun_out/inc/ &&
VARIANTS="-;DML_MERGE_AT=$R1;DML_MERGE_AT=$R2" ROUNDS=2 BENCH_ARGS="--models ResNet50 --no-service" \
  bash tools/gpu_env_ab.sh
