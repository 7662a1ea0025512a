# round-3: kernel-trace profiles of the single-model pipelines + per-op times (roofline inputs)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && export DML_SKIP_BUILD=1 && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3e_r50 -o run -- python3 $R/bench.py --models ResNet50 --no-service --steps 30 > $R/gpurun_out/r3e_r50.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3e_inc -o run -- python3 $R/bench.py --models InceptionV3 --no-service --steps 30 > $R/gpurun_out/r3e_inc.log 2>&1 && \
cd $R && timeout -k 10 300 python3 bench.py --models ResNet50,InceptionV3 --no-service --steps 60 --op-times gpurun_out/r3e_op_times.json > gpurun_out/r3e_optimes.log 2>&1
