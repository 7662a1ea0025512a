#!/bin/bash
# Full re-tune A/B: bench on the committed table (tag c4la), bench that re-times
# every shape under the new tag, bench on the new table, the old table again.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 900 python bench.py --steps 30 --warmup 5 > gpurun_out/rt_$n.log 2>&1 \
    && echo "$n: $(tail -1 gpurun_out/rt_$n.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["models"]["InceptionV3"]["value"], d["verified_top5"])')" \
    || { tail -20 gpurun_out/rt_$n.log; exit 1; }
}
run old1 DML_TUNING_TAG=c4la
run tune DML_TUNING_TAG=c5rt
run new1 DML_TUNING_TAG=c5rt
run old2 DML_TUNING_TAG=c4la
run new2 DML_TUNING_TAG=c5rt
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/conv_tuning_rt.json
