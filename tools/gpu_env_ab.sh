#!/bin/bash
# Interleaved env-variant A/B of bench.py on one box: ROUNDS x VARIANTS (';'-separated
# env assignments, "-" = defaults), one bench line each -> gpurun_out/envab_<i>_r<r>.log.
#   VARIANTS="-;DML_CHAIN=2;DML_CHAIN_C256=1" ROUNDS=2 BENCH_ARGS="--models ResNet50 --no-service" bash tools/gpu_env_ab.sh
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS:--}"
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for v in "${VS[@]}"; do
    i=$((i+1))
    envs=()
    [ "$v" != "-" ] && read -ra envs <<< "$v"
    env "${envs[@]}" timeout -k 10 300 python bench.py --steps ${STEPS:-60} --warmup 5 ${BENCH_ARGS:-} \
      > gpurun_out/envab_${i}_r$r.log 2>&1 || { tail -20 gpurun_out/envab_${i}_r$r.log; exit 1; }
    echo "round $r [$v]: $(tail -1 gpurun_out/envab_${i}_r$r.log | grep -o '"value": [0-9.]*' | head -1)"
  done
done
