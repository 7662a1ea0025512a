#!/bin/bash
# Stem probes + InceptionV3 / ResNet50 sub-batch split variants (bench.py --splits/--streams).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/stem_bench.py --lib ${LIBS:-variants/libdml_stemconvonly.so,variants/libdml_stemnold.so} \
  --out gpurun_out/stem_bench2.json > gpurun_out/stem_bench2.log 2>&1 && grep -v amdgpu.ids gpurun_out/stem_bench2.log || exit 1
for v in ${VARIANTS:-"InceptionV3:2:0" "InceptionV3:4:2" "InceptionV3:4:4" "InceptionV3:2:0"}; do
  IFS=: read m sp st <<< "$v"
  timeout -k 10 300 python -u bench.py --model $m --steps 30 --warmup 5 --no-service --splits $sp --streams $st \
    > gpurun_out/split_${m}_${sp}_${st}.log 2>&1 || { tail -20 gpurun_out/split_${m}_${sp}_${st}.log; exit 1; }
  echo "$m splits $sp streams $st: $(grep '"metric"' gpurun_out/split_${m}_${sp}_${st}.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done
