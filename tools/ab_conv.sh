#!/bin/bash
# A/B of two native libraries on the conv layer shapes (same box, same process
# order base,new,new,base): DML_LIB=<variant .so> python tools/conv_bench.py ...
#   BASE=build/ab/libdml_base.so MODEL=ResNet50 BATCH=128 CFGS=11,14,... tools/ab_conv.sh
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
BASE=${BASE:-build/ab/libdml_base.so}
NEW=${NEW:-distributed_machine_learning_amd/libdml_hip.so}
MODEL=${MODEL:-ResNet50}; BATCH=${BATCH:-128}; CFGS=${CFGS:-11,14,15,22,24,26,27}
i=0
for lib in $BASE $NEW $NEW $BASE; do
  i=$((i+1))
  DML_LIB=$lib timeout -k 10 300 python tools/conv_bench.py --model $MODEL --batch $BATCH --cfgs $CFGS --iters 20 \
    --out gpurun_out/ab/run$i.json > gpurun_out/ab/run$i.log 2>&1 || { tail -20 gpurun_out/ab/run$i.log; exit 1; }
  tail -1 gpurun_out/ab/run$i.log | cut -c1-300
done
