#!/bin/bash
# Cold-cache tuning A/B: bench on the committed (warm-timed) table, bench that
# re-times every shape cold (DML_TUNE_COLD=1, tag c5cold), then both again.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 900 python bench.py --steps 30 --warmup 5 > gpurun_out/ct_$n.log 2>&1 \
    && echo "$n: $(tail -1 gpurun_out/ct_$n.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["models"]["InceptionV3"]["value"], d["verified_top5"])')" \
    || { tail -20 gpurun_out/ct_$n.log; exit 1; }
}
run warm1 DML_TUNING_TAG=c5rt
run tune DML_TUNING_TAG=c5cold DML_TUNE_COLD=1
run cold1 DML_TUNING_TAG=c5cold
run warm2 DML_TUNING_TAG=c5rt
run cold2 DML_TUNING_TAG=c5cold
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/conv_tuning_ct.json
