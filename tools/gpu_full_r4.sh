#!/bin/bash
# Full GPU suite + smoke (what the driver runs at round end), then the r4 A/B round.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_suite.log 2>&1; rc=$?
tail -4 gpurun_out/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || exit 1
[ -n "$NO_AB" ] || bash tools/gpu_ab_r4.sh
