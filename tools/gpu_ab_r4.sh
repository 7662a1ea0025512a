#!/bin/bash
# r4 A/B round: register-staged operand probes (conv_ab.py, bit-identical outputs required), then
# stem probes + InceptionV3 split variants (gpu_split_ab.sh).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in ${AB_LIBS:-wreg xreg}; do
  timeout -k 10 400 python -u tools/conv_ab.py --lib variants/libdml_$v.so --out gpurun_out/conv_ab_$v.json \
    > gpurun_out/conv_ab_$v.log 2>&1; rc=$?
  echo "== $v (rc $rc)"; grep -v amdgpu.ids gpurun_out/conv_ab_$v.log | tail -14
  [ $rc -le 1 ] || exit $rc
done
[ -n "$NO_SPLIT" ] || bash tools/gpu_split_ab.sh
