mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_rr_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rr_pytest.log 2>&1 || { tail -20 gpurun_out/rr_pytest.log; exit 1; }
tail -1 gpurun_out/rr_pytest.log
timeout -k 10 300 python -u tools/conv_ws_ab.py --shapes r50_3x3_s2 --ws 150,151,152 --out gpurun_out/rr_ab.json > gpurun_out/rr_ab.log 2>&1 || { tail -20 gpurun_out/rr_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rr_ab.log | tail -2
timeout -k 10 120 python -u tools/rr_stamps.py --cfg 150 > gpurun_out/rr_stamps.log 2>&1 || exit 1
for th in "" "100000,50,1000"; do
  DML_GC_THRESHOLD=$th timeout -k 10 600 python -u tools/store_capacity.py --world 8 --rate 370 --batches-per-rank 1200 --out gpurun_out/storecap_gc$th.json > gpurun_out/storecap_gc$th.log 2>&1; echo "storecap [$th] rc=$?"; grep CAPACITY gpurun_out/storecap_gc$th.log
done
ADD=150,151,152 STEPS=20 bash tools/gpu_ws_tune.sh
