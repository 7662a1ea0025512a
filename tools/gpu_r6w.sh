#!/bin/bash
# r6 call W: persistent conv3x3+pool(+1x1) kernel (DML_CPOOL_PERSIST=1) vs the one-block-per-
# workgroup kernel: numerics, then InceptionV3 per-op times (64-image sub-batch) both ways, twice.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6_w
mkdir -p $O
export TMPDIR=/tmp
DML_CPOOL_PERSIST=1 timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py -x -q -k "pool" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 0 1; do
    DML_CPOOL_PERSIST=$v timeout -k 10 300 python tools/op_times.py --runs InceptionV3:64 --out-dir $O/ops_p${v}_r$r > $O/ops_p${v}_r$r.log 2>&1 || { tail -10 $O/ops_p${v}_r$r.log; exit 1; }
    python - <<PY
import json
r = json.load(open("$O/ops_p${v}_r$r/op_times_InceptionV3_b64.json"))
cp = [(n, t) for n, t in r["ops"] if "conv2d_3" in n]
print("persist=$v r$r total %.3f ms" % r["total_ms"], [(n, round(t * 1e3, 1)) for n, t in cp])
PY
  done
done
