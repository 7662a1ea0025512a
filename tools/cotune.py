"""Joint tile-config tuning of the co-scheduled sub-batch plans of a SplitEngine.

ops/tuning.py picks each conv's tile config by timing it ALONE. In the serving
step two sub-batch graphs run concurrently on two streams, so a config that is
fastest alone (e.g. many small tiles that fill every CU) is not necessarily
best next to the other stream's kernels. This tool does a greedy coordinate
descent over the conv ops: for each op it tries the K configs that were
fastest alone, re-points BOTH sub-batch plans at each (dml_plan_set_cfg),
re-captures the hipGraphs and times the whole split forward; a change is kept
only if it beats the current forward by more than --thresh.

  python tools/cotune.py [--model ResNet50] [--batch 256] [--cands 3] [--out f.json]
Prints progress lines and one final JSON line {layer: cfg} + before/after ms.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_machine_learning_amd import _native as N  # noqa: E402
from distributed_machine_learning_amd.models import build_model, canonical_name  # noqa: E402
from distributed_machine_learning_amd.models.engine import SplitEngine  # noqa: E402
from distributed_machine_learning_amd.models.graph import Conv, Dense, FusedConv  # noqa: E402
from distributed_machine_learning_amd.ops import tuning  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="ResNet50")
ap.add_argument("--batch", type=int, default=0)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--cands", type=int, default=3)
ap.add_argument("--thresh", type=float, default=0.004)
ap.add_argument("--budget_s", type=float, default=240.0)
ap.add_argument("--out", default="")
args = ap.parse_args()

model = canonical_name(args.model)
B = args.batch or {"ResNet50": 256, "InceptionV3": 128}[model]
g, w = build_model(model, seed=0, calibrate=False)
se = SplitEngine(g, w, batch=B, splits=2, src_slots=1)
L = N.lib()
main = torch.cuda.Stream()
sp = N.stream_ptr(main)
plans = [e.plans[0] for e in se.engines]
e0 = se.engines[0]
nodes = {n.name: n for n in e0.g.nodes}


def forward_ms() -> float:
    for p in plans:
        N.check(L.dml_plan_capture(p, sp), "capture")
    for e in se.engines:
        e.graph_captured[0] = True
    se.run(main, use_graph=True)
    main.synchronize()
    vals = []
    for _ in range(args.reps):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record(main)
        for _ in range(args.iters):
            se.run(main, use_graph=True)
        e.record(main)
        e.synchronize()
        vals.append(s.elapsed_time(e) / args.iters)
    vals.sort()
    return vals[len(vals) // 2]


t_start = time.time()
base = forward_ms()
cur = base
print(f"baseline split forward {base:.3f} ms", flush=True)
changes = {}
table = {}  # the changes as tuning-table entries (shape key -> cfg; shared shapes: last change wins)
for i, name in enumerate(e0.op_names):
    if time.time() - t_start > args.budget_s:
        print("time budget reached", flush=True)
        break
    c0 = L.dml_plan_get_cfg(plans[0], i)
    n = nodes.get(name)
    if c0 < 0 or not isinstance(n, (Conv, Dense, FusedConv)):
        continue
    a = e0._conv_args(n)
    alone = []
    for c in tuning.valid_cfgs(a):
        try:
            alone.append((tuning.time_cfg(a, c), c))
        except N.NativeError:
            pass
    alone.sort()
    cands = [c for _, c in alone if c != c0][: args.cands]
    best = (cur, c0)
    for c in cands:
        if any(L.dml_plan_set_cfg(p, i, c) < 0 for p in plans):
            continue
        t = forward_ms()
        if t < best[0]:
            best = (t, c)
    for p in plans:
        L.dml_plan_set_cfg(p, i, best[1] if best[0] < cur * (1 - args.thresh) else c0)
    if best[0] < cur * (1 - args.thresh):
        changes[name] = best[1]
        table[tuning.shape_key(a)] = best[1]
        print(f"{name}: cfg {c0} -> {best[1]}  {cur:.3f} -> {best[0]:.3f} ms", flush=True)
        cur = best[0]
final = forward_ms()
res = {"model": model, "batch": B, "baseline_ms": round(base, 4), "final_ms": round(final, 4), "changes": changes,
       "table": table}
print(json.dumps(res), flush=True)
if args.out:
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
