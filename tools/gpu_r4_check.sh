#!/bin/bash
# r4 iteration: stem / serving GPU tests, stem microbench, service depth sweep + full bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_stem_gpu.py tests/test_serving_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "${TESTS_K:-stem or pool or index_table or world1_outputs or store_images}" \
  > gpurun_out/r4_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/stem_bench.py --out gpurun_out/stem_bench.json > gpurun_out/stem_bench.log 2>&1 \
  && grep -v amdgpu.ids gpurun_out/stem_bench.log || exit 1
[ -n "$NO_SVC" ] || DEPTHS="${DEPTHS:-4 8}" bash tools/gpu_svc_depth.sh
