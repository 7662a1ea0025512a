#!/bin/bash
# Pipeline-level co-tuning (tools/cotune_pipe.py) on the committed table, merged
# into a copy, then bench A/B (three interleaved rounds).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=distributed_machine_learning_amd/tuning/conv_tuning.json
cp $T /tmp/tuning_base.json
for m in ${MODELS:-ResNet50}; do
  timeout -k 10 700 python -u tools/cotune_pipe.py --model $m ${COTUNE_ARGS:-} --out gpurun_out/cotp_$m.json > gpurun_out/cotp_$m.log 2>&1 \
    && tail -1 gpurun_out/cotp_$m.log | cut -c1-400 || { tail -20 gpurun_out/cotp_$m.log; exit 1; }
done
python - <<'PY'
import json, os
t = json.load(open("/tmp/tuning_base.json"))
for m in os.environ.get("MODELS", "ResNet50").split():
    t.update(json.load(open(f"gpurun_out/cotp_{m}.json"))["table"])
json.dump(dict(sorted(t.items())), open("/tmp/tuning_co.json", "w"), indent=0)
json.dump(dict(sorted(t.items())), open("gpurun_out/conv_tuning_cotp.json", "w"), indent=0)
PY
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 600 python bench.py --steps 30 --warmup 5 > gpurun_out/cp_$n.log 2>&1 \
    && echo "$n: $(tail -1 gpurun_out/cp_$n.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["models"]["InceptionV3"]["value"], d["verified_top5"])')" \
    || { tail -20 gpurun_out/cp_$n.log; exit 1; }
}
for rnd in 1 2 3; do
  run base$rnd DML_TUNING_CACHE=/tmp/tuning_base.json
  run co$rnd DML_TUNING_CACHE=/tmp/tuning_co.json
done
