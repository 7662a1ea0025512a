#!/bin/bash
# Interleaved tuning-table A/B of bench.py on one box: ROUNDS x TABLES (space-separated JSON
# paths, each used as DML_TUNING_CACHE), one bench line each -> gpurun_out/tab_<i>_r<r>.log.
#   TABLES="ab_tables/a.json ab_tables/b.json" ROUNDS=3 STEPS=200 BENCH_ARGS="--model InceptionV3 --no-service"
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
read -ra TS <<< "${TABLES}"
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for t in "${TS[@]}"; do
    i=$((i+1))
    cp "$t" /tmp/tab_$i.json
    DML_TUNING_CACHE=/tmp/tab_$i.json timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} \
      > gpurun_out/tab_${i}_r$r.log 2>&1 || { tail -20 gpurun_out/tab_${i}_r$r.log; exit 1; }
    echo "round $r [$t]: $(grep -o '"value": [0-9.]*' gpurun_out/tab_${i}_r$r.log | tr '\n' ' ')"
  done
done
