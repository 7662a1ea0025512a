#!/bin/bash
# Sweep bench.py over sub-batch splits / streams for one model.
# usage: MODEL=InceptionV3 SWEEP="1:1 2:2 4:2" tools/gpu_sweep.sh
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
for ss in ${SWEEP:-1:1 2:2}; do
  sp=${ss%%:*}; st=${ss##*:}
  f=gpurun_out/sweep/${MODEL:-InceptionV3}_s${sp}_t${st}.log
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --models ${MODEL:-InceptionV3} --splits $sp --streams $st \
    ${BENCH_ARGS:-} > $f 2>&1 || { tail -20 $f; exit 1; }
  python - "$f" "$sp" "$st" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"splits {sys.argv[2]} streams {sys.argv[3]}: {d['value']:.1f} img/s p50 {d['p50_latency_ms']} ms")
PY
done

