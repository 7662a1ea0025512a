#!/bin/bash
# r6 call V: the one-call native batch launch (dml_launch_seq): the service GPU tests (rows
# checked against Engine.infer), then the distinct pass and the synthetic service with
# DML_NATIVE_LAUNCH=1 / 0, interleaved twice.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_rank_service_gpu.py tests/test_serving_gpu.py -x -q --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 1 0; do
    DML_NATIVE_LAUNCH=$v timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/distinct_n${v}_r$r.log 2>&1 || { tail -20 $O/distinct_n${v}_r$r.log; exit 1; }
    echo "native=$v r$r $(python tools/bench_summary.py $O/distinct_n${v}_r$r.log | sed 's/.*ResNet50 [0-9]*//')"
    grep -o '"loop_phase_s": {[^}]*}' $O/distinct_n${v}_r$r.log | tail -1
  done
done
