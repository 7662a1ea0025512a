#!/bin/bash
# Channel-padded conv input probe (tools/cinpad_probe.py)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/cinpad_probe.py --iters 20 > gpurun_out/cinpad.log 2>&1
rc=$?
cat gpurun_out/cinpad.log
exit $rc
