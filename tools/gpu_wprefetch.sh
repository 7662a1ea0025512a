#!/bin/bash
# Weight-prefetch ops (DML_WPREFETCH=<min weight bytes>) A/B, interleaved, on one box.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 900 python bench.py --steps 30 --warmup 5 > gpurun_out/wp_$n.log 2>&1 \
    && echo "$n: $(tail -1 gpurun_out/wp_$n.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["models"]["InceptionV3"]["value"], d["verified_top5"])')" \
    || { tail -20 gpurun_out/wp_$n.log; exit 1; }
}
run off1 DML_WPREFETCH=0
run 1m_1 DML_WPREFETCH=1048576
run 512k_1 DML_WPREFETCH=524288
run off2 DML_WPREFETCH=0
run 1m_2 DML_WPREFETCH=1048576
run 512k_2 DML_WPREFETCH=524288
DML_WPREFETCH=1048576 timeout -k 10 600 python bench.py --steps 5 --warmup 2 --models ResNet50 --op-times gpurun_out/wp_op_times.json > gpurun_out/wp_ops.log 2>&1 || { tail -20 gpurun_out/wp_ops.log; exit 1; }
