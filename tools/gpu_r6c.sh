#!/bin/bash
# r6 call C: the 51,200-distinct store-image pass with the 24 GiB plane cache (GPU decodes vs
# plane reuse counted), then the world-8 output-store capacity offered 600 batches/s per rank.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > gpurun_out/distinct51200_c.log 2>&1 || { tail -20 gpurun_out/distinct51200_c.log; exit 1; }
python tools/bench_summary.py gpurun_out/distinct51200_c.log
grep -o '"gpu_jpeg_decodes_coordinator": [0-9]*, "gpu_plane_reuse_coordinator": [0-9]*' gpurun_out/distinct51200_c.log || true
timeout -k 10 600 python tools/store_capacity.py --world 8 --rate 600 --batches-per-rank 600 --out gpurun_out/capacity_w8_600.json > gpurun_out/capacity_w8_600.log 2>&1 || { tail -20 gpurun_out/capacity_w8_600.log; exit 1; }
grep -E 'CAPACITY' gpurun_out/capacity_w8_600.log; python -c "
import json; d=json.load(open('gpurun_out/capacity_w8_600.json')); c=d['capacity']
print('batches/s', c['batches_per_s'], 'per rank', c['batches_per_s_per_rank'], 'backend idle', c['backend_idle_s_per_rank'], 'span', c['backend_span_s_per_rank'][:2])"
