#!/bin/bash
# r6 call A: GPU JPEG numerics with the parallel Huffman decode, its per-window A/B against the
# serial one, the short-run (driver's 20 steps) vs 200-step bench and a spin-up variant, then a
# rocprofv3 kernel trace of the driver's exact bench command.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py tests/test_resize_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/jpeg_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/jpeg_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/jpeg_bench.py > gpurun_out/jpeg_par.log 2>&1 && cat gpurun_out/jpeg_par.log | grep -v amdgpu.ids || exit 1
DML_JPEG_SERIAL=1 timeout -k 10 300 python -u tools/jpeg_bench.py > gpurun_out/jpeg_ser.log 2>&1 && cat gpurun_out/jpeg_ser.log | grep -v amdgpu.ids || exit 1
for r in 1 2; do
  for m in InceptionV3 ResNet50; do
    for v in "20" "200" "20 spin"; do
      set -- $v
      env DML_BENCH_SPINUP_S=$([ "$2" = spin ] && echo 1.0 || echo 0) timeout -k 10 300 python bench.py --model $m --no-service --steps $1 --warmup 5 > gpurun_out/short_${m}_$1_$2_r$r.log 2>&1 || { tail -20 gpurun_out/short_${m}_$1_$2_r$r.log; exit 1; }
      echo "r$r $m steps=$1 ${2:-} $(grep -o '"value": [0-9.]*' gpurun_out/short_${m}_$1_$2_r$r.log | head -1)"
    done
  done
done
if [ -n "$PROFILE" ]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_driver -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_driver.log 2>&1 && echo profiled && tail -1 $GRAFT_REPO_ROOT/gpurun_out/prof_driver.log | cut -c1-300 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_driver.log; exit 1; }
fi
