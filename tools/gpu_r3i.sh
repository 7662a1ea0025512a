# round-3: full GPU test suite, the driver's default bench line, smoke; tuning cache back
set -o pipefail
cd $GRAFT_REPO_ROOT
export DML_SKIP_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3i_pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/r3i_pytest_gpu.log
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/r3i_conv_tuning_after_tests.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r3i_bench.log 2>&1 && tail -1 gpurun_out/r3i_bench.log | cut -c1-400 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/r3i_smoke.log 2>&1 && tail -3 gpurun_out/r3i_smoke.log
cp distributed_machine_learning_amd/tuning/conv_tuning.json gpurun_out/r3i_conv_tuning.json
