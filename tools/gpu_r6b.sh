#!/bin/bash
# r6 call B: the driver's exact bench command (twice), then the 51,200-distinct store-image pass.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/jpeg_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/jpeg_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/jpeg_bench.py > gpurun_out/jpeg_par64.log 2>&1 && grep -v amdgpu.ids gpurun_out/jpeg_par64.log || exit 1
for r in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver_cmd_r$r.log 2>&1 || { tail -20 gpurun_out/driver_cmd_r$r.log; exit 1; }
  python tools/bench_summary.py gpurun_out/driver_cmd_r$r.log 2>/dev/null || tail -1 gpurun_out/driver_cmd_r$r.log | cut -c1-400
done
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > gpurun_out/distinct51200.log 2>&1 || { tail -20 gpurun_out/distinct51200.log; exit 1; }
python tools/bench_summary.py gpurun_out/distinct51200.log 2>/dev/null || tail -1 gpurun_out/distinct51200.log | cut -c1-600
# fresh per-op rooflines of the final table (one forward per model, per-op event timing)
for m in ResNet50 InceptionV3; do
  timeout -k 10 300 python bench.py --model $m --no-service --steps 20 --warmup 5 --op-times gpurun_out/op_times_$m.json > gpurun_out/optimes_$m.log 2>&1 || { tail -20 gpurun_out/optimes_$m.log; exit 1; }
  python tools/roofline.py gpurun_out/op_times_$m.json --model $m --out gpurun_out/roofline_$m.csv | tail -2
done
# output-store capacity at world 8 on the box's CPUs (no GPU): 470 batches/s per rank offered
timeout -k 10 600 python tools/store_capacity.py --world 8 --rate 470 --batches-per-rank 300 --out gpurun_out/capacity_w8.json > gpurun_out/capacity_w8.log 2>&1 || { tail -20 gpurun_out/capacity_w8.log; exit 1; }
grep -E '"batches_per_s"|CAPACITY' gpurun_out/capacity_w8.log | cut -c1-300
python tools/output_path_ab.py --threads 4 --out gpurun_out/output_path_ab_box.json | tail -4
