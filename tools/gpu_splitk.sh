set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "split_k or chunk_major or non_tile" > gpurun_out/pytest_splitk.log 2>&1 || { tail -30 gpurun_out/pytest_splitk.log; exit 1; }
tail -1 gpurun_out/pytest_splitk.log
timeout -k 10 600 python bench.py --steps 30 --warmup 5 --op-times gpurun_out/op_times.json > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-250 || { tail -30 gpurun_out/bench.log; exit 1; }
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/conv_tuning.json
