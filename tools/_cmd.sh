#!/bin/bash
# scratch gpurun command for the current A/B (overwritten per experiment)
set -o pipefail
mkdir -p gpurun_out
PROFILE=1 STEPS=30 bash tools/gpu_round.sh &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log
