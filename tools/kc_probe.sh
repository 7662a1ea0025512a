set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/conv_bench.py --model ResNet50 --batch 128 --only _2_conv --cfgs 10,11,14,15,17,26,28,30,31,34 --kchunk 64 --out gpurun_out/kc_r50.json > gpurun_out/kc_r50.log 2>&1 && \
timeout -k 10 400 python tools/conv_bench.py --model InceptionV3 --batch 64 --cfgs 11,14,15,23,26,28,30,31,34 --kchunk 64 --out gpurun_out/kc_inc.json > gpurun_out/kc_inc.log 2>&1
rc=$?; tail -3 gpurun_out/kc_r50.log gpurun_out/kc_inc.log; exit $rc
