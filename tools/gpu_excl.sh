#!/bin/bash
# A/B: committed table vs a cold re-tune that excludes the one-workgroup-per-CU
# tiles (LDS > 80 KiB: 10, 13, 16, 17, 21, 34, 37) under tag c5x1.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 900 python bench.py --steps 30 --warmup 5 > gpurun_out/ex_$n.log 2>&1 \
    && echo "$n: $(tail -1 gpurun_out/ex_$n.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["models"]["InceptionV3"]["value"], d["verified_top5"])')" \
    || { tail -20 gpurun_out/ex_$n.log; exit 1; }
}
X="DML_TUNING_TAG=c5x1 DML_TUNE_EXCLUDE=10,13,16,17,21,34,37"
run tune $X
for rnd in 1 2 3; do
  run base$rnd DML_TUNING_TAG=c5cold
  run x$rnd $X
done
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/conv_tuning_x.json
