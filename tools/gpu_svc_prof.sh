#!/bin/bash
# Service-path kernel census: GPU serving tests (TESTS_K selects), then a kernel-trace
# rocprofv3 run of tools/serve_bench.py (world 1) and the per-kernel summary of it —
# which kernels the serving launch path runs (no gather / copy kernels expected).
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS_K" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_serving_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread \
    -k "$TESTS_K" > gpurun_out/svc_tests.log 2>&1; rc=$?
  grep -E "PASS|FAIL|Error" gpurun_out/svc_tests.log | tail -20
  [ $rc -eq 0 ] || exit $rc
fi
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_svc -o svc -- \
  python3 $R/tools/serve_bench.py --resnet-images ${RI:-25600} --inception-images ${II:-12800} \
  > $R/gpurun_out/prof_svc.log 2>&1 || { tail -30 $R/gpurun_out/prof_svc.log; exit 1; }
grep '"metric"' $R/gpurun_out/prof_svc.log | cut -c1-600
python3 $R/tools/kernel_census.py $R/gpurun_out/prof_svc > $R/gpurun_out/prof_svc_census.txt && cat $R/gpurun_out/prof_svc_census.txt | head -40
