#!/bin/bash
# Non-temporal activation DMA for 1x1 convs: the batch-rows test under both settings, then
# interleaved bench rounds DML_XNT=1 (default) vs 0.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for x in 0 1 0 1; do
  DML_XNT=$x timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -q --timeout 240 --timeout-method thread \
    -k "batch_rows_independent" > gpurun_out/xnt_rows_$x.log 2>&1
  echo "xnt $x rows test: $(tail -1 gpurun_out/xnt_rows_$x.log)"
done
for r in 1 2; do
  for x in 1 0; do
    for m in ResNet50 InceptionV3; do
      DML_XNT=$x timeout -k 10 300 python -u bench.py --model $m --steps 30 --warmup 5 --no-service \
        > gpurun_out/xnt_${x}_${m}_$r.log 2>&1 || { tail -20 gpurun_out/xnt_${x}_${m}_$r.log; exit 1; }
      echo "xnt $x $m round $r: $(grep '"metric"' gpurun_out/xnt_${x}_${m}_$r.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
    done
  done
done
