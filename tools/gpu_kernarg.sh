#!/bin/bash
# HIP_FORCE_DEV_KERNARG A/B on both models, interleaved, four rounds.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 600 python bench.py --steps 30 --warmup 5 > gpurun_out/ka_$n.log 2>&1 \
    && echo "$n: $(tail -1 gpurun_out/ka_$n.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["models"]["InceptionV3"]["value"], d["verified_top5"])')" \
    || { tail -20 gpurun_out/ka_$n.log; exit 1; }
}
for rnd in 1 2 3 4; do
  run base$rnd HIP_FORCE_DEV_KERNARG=0
  run ka$rnd HIP_FORCE_DEV_KERNARG=1
done
