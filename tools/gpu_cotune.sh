#!/bin/bash
# In-situ co-tuning (tools/cotune.py: each conv's candidates timed inside the
# two-stream split forward) on top of the committed cold-tuned table, merged
# into a copy of the table, then bench A/B: committed table vs co-tuned copy.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=distributed_machine_learning_amd/tuning/conv_tuning.json
cp $T /tmp/tuning_base.json
for m in ${MODELS:-ResNet50 InceptionV3}; do
  timeout -k 10 600 python -u tools/cotune.py --model $m --budget_s 400 ${COTUNE_ARGS:-} --out gpurun_out/cotune_$m.json > gpurun_out/cotune_$m.log 2>&1 \
    && tail -1 gpurun_out/cotune_$m.log | cut -c1-300 || { tail -20 gpurun_out/cotune_$m.log; exit 1; }
done
python - <<'PY'
import json
t = json.load(open("/tmp/tuning_base.json"))
import os
for m in os.environ.get("MODELS", "ResNet50 InceptionV3").split():
    t.update(json.load(open(f"gpurun_out/cotune_{m}.json"))["table"])
json.dump(dict(sorted(t.items())), open("/tmp/tuning_co.json", "w"), indent=0)
json.dump(dict(sorted(t.items())), open("gpurun_out/conv_tuning_co.json", "w"), indent=0)
PY
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 600 python bench.py --steps 30 --warmup 5 > gpurun_out/co_$n.log 2>&1 \
    && echo "$n: $(tail -1 gpurun_out/co_$n.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["models"]["InceptionV3"]["value"], d["verified_top5"])')" \
    || { tail -20 gpurun_out/co_$n.log; exit 1; }
}
for rnd in 1 2 3; do
  run base$rnd DML_TUNING_CACHE=/tmp/tuning_base.json
  run co$rnd DML_TUNING_CACHE=/tmp/tuning_co.json
done
