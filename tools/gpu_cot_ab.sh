#!/bin/bash
# Co-tuned table (variants/conv_tuning_cot.json) vs the shipped one, MODEL (default InceptionV3), interleaved rounds.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2 3; do
  for t in base cot; do
    log=gpurun_out/cot_${MODEL:-InceptionV3}_${t}_$r.log
    tab=distributed_machine_learning_amd/tuning/conv_tuning.json; [ $t = cot ] && tab=variants/conv_tuning_cot.json
    DML_TUNING_CACHE=$tab timeout -k 10 300 python -u bench.py --model ${MODEL:-InceptionV3} --steps 30 --warmup 5 --no-service \
      > $log 2>&1 || { tail -20 $log; exit 1; }
    echo "$t round $r: $(grep '"metric"' $log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["verified_top5"])')"
  done
done
