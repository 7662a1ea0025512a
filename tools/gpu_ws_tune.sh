#!/bin/bash
# One gpurun call: adopt the warp-specialised tiles into the tuning table (DML_TUNE_ADD: a
# cached shape switches only when a new tile is >= 3 % faster cold), then interleaved bench
# rounds of the new table against the committed one on the same box; the table comes back
# in gpurun_out/. Also the output-store capacity harness (CPU only, world 8).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
cp distributed_machine_learning_amd/tuning/conv_tuning.json /tmp/table_old.json
ADD=${ADD:-100,101,102,103,104,105,106,107,108,109,110,111,112,120,121,122,123,124,125,126,127,128,129}
STEPS=${STEPS:-20}
DML_TUNE_ADD=$ADD timeout -k 10 900 python -u bench.py --steps $STEPS --warmup 5 --no-service > gpurun_out/tune_bench.log 2>&1 || { tail -30 gpurun_out/tune_bench.log; exit 1; }
python tools/bench_summary.py gpurun_out/tune_bench.log
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/conv_tuning_new.json
for r in 1 2; do
  DML_TUNING_CACHE=/tmp/table_old.json timeout -k 10 600 python -u bench.py --steps $STEPS --warmup 5 --no-service > gpurun_out/ab_old_$r.log 2>&1 || { tail -30 gpurun_out/ab_old_$r.log; exit 1; }
  python tools/bench_summary.py gpurun_out/ab_old_$r.log
  timeout -k 10 600 python -u bench.py --steps $STEPS --warmup 5 --no-service > gpurun_out/ab_new_$r.log 2>&1 || { tail -30 gpurun_out/ab_new_$r.log; exit 1; }
  python tools/bench_summary.py gpurun_out/ab_new_$r.log
done
if [ -n "$STORECAP" ]; then
  timeout -k 10 600 python -u tools/store_capacity.py --world 8 --rate 370 --batches-per-rank 300 --out gpurun_out/store_capacity_box.json > gpurun_out/store_capacity_box.log 2>&1; echo "storecap rc=$?"; head -1 gpurun_out/store_capacity_box.log | cut -c1-400
fi
