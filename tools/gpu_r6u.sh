#!/bin/bash
# r6 call U: the result gather's RCCL branch alone at world 1.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6_u
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/probe_result_gather.py > gpurun_out/r6_u/probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6_u/probe.log | tail -30
exit $rc
