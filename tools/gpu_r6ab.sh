#!/bin/bash
# r6 call AB (final tree): the full GPU suite, the driver's bench command, the 51,200-distinct pass twice.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_final4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python tools/bench_summary.py $O/bench.log
for r in 1; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --models ResNet50 --svc-store-images 51200 --kill-pass off > $O/distinct_r$r.log 2>&1 || { tail -20 $O/distinct_r$r.log; exit 1; }
  python tools/bench_summary.py $O/distinct_r$r.log
done
