# round-3: chained stage-3 boundaries in the pipeline: base / 4-wave / 8-wave, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export DML_SKIP_BUILD=1
mkdir -p gpurun_out
B="python -u bench.py --models ResNet50 --no-service --steps 100"
timeout -k 10 300 $B > gpurun_out/r3h_base1.log 2>&1 && \
DML_CHAIN=1 timeout -k 10 300 $B > gpurun_out/r3h_c4a.log 2>&1 && \
DML_CHAIN=1 DML_CHAIN_WAVES=8 timeout -k 10 300 $B > gpurun_out/r3h_c8a.log 2>&1 && \
timeout -k 10 300 $B > gpurun_out/r3h_base2.log 2>&1 && \
DML_CHAIN=1 timeout -k 10 300 $B > gpurun_out/r3h_c4b.log 2>&1 && \
DML_CHAIN=1 DML_CHAIN_WAVES=8 timeout -k 10 300 $B > gpurun_out/r3h_c8b.log 2>&1
