#!/bin/bash
# v2 K-loop probes 5 (no per-lane K walk) and 6 (no K-loop barrier) vs the main build, per layer
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in p5 p6; do
  timeout -k 10 300 python -u tools/conv_ab.py --lib variants/libdml_$v.so --cfgs 11,14,15,24,38 --iters 20 \
    --out gpurun_out/conv_ab_v2probe_$v.json > gpurun_out/conv_ab_v2probe_$v.log 2>&1
  rc=$?
  echo "== $v rc $rc"; cat gpurun_out/conv_ab_v2probe_$v.log
  [ $rc -le 1 ] || exit $rc
done
