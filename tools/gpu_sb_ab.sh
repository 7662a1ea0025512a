#!/bin/bash
# Concurrent collective-service bench twice + the ResNet50 bench twice (A/B helper).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
for i in 1 2; do
  timeout -k 10 300 python tools/serve_bench.py --resnet-images 40960 --inception-images 20480 > gpurun_out/ab/sb_$i.log 2>&1 || { tail -20 gpurun_out/ab/sb_$i.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/ab/sb_$i.log').read().strip().splitlines()[-1]); print('service', d['value'], d['resnet50_images_per_s'], d['inceptionv3_images_per_s'], d['p50_latency_ms'])"
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/ab/bench_$i.log 2>&1 || { tail -20 gpurun_out/ab/bench_$i.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/ab/bench_$i.log').read().strip().splitlines()[-1]); print('bench', d['value'], d['models']['InceptionV3']['value'])"
done
