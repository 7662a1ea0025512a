"""Co-tuning inside the serving pipeline (the loop bench.py times).

tools/cotune.py scores a tile change by the split forward alone; in the serving
pipeline consecutive batches overlap (the next batch's sub-batch streams start
on their own input events), so a tile that hogs LDS at the end of batch k also
slows the head of batch k+1. This tool times ``ServingPipeline.run`` itself: for
each conv op it tries the best-alone candidates (ops/tuning.time_cfg, cold) —
for a grouped launch every other grouped tile — on every plan of both sub-batch engines, re-captures the graphs and keeps a change
only if the pipeline's ms/step improves by more than --thresh. Prints one final
JSON line whose "table" holds the changes as tuning-table entries.

  python tools/cotune_pipe.py [--model ResNet50] [--cands 3] [--out f.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_machine_learning_amd import _native as N  # noqa: E402
from distributed_machine_learning_amd.models import build_model, canonical_name  # noqa: E402
from distributed_machine_learning_amd.models.engine import SplitEngine  # noqa: E402
from distributed_machine_learning_amd.models.graph import Conv, Dense, FusedConv, Pool  # noqa: E402
from distributed_machine_learning_amd.ops import tuning  # noqa: E402
from distributed_machine_learning_amd.parallel.dataplane import DESC_FIELDS, DataPlane, init_process_group  # noqa: E402
from distributed_machine_learning_amd.parallel.pipeline import ServingPipeline  # noqa: E402
from distributed_machine_learning_amd.parallel.staging import PinnedImageStore  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="ResNet50")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--cands", type=int, default=3)
ap.add_argument("--thresh", type=float, default=0.004)
ap.add_argument("--budget_s", type=float, default=400.0)
ap.add_argument("--out", default="")
args = ap.parse_args()

model = canonical_name(args.model)
B = {"ResNet50": 256, "InceptionV3": 128}[model]
rank, world, local = init_process_group()
dev = torch.device("cuda", local)
g, w = build_model(model, seed=0, calibrate=False)
se = SplitEngine(g, w, batch=B, device=str(dev), src_slots=2, splits=2)
store = PinnedImageStore(capacity=4 * B, hw=g.input_hw)
store.fill_synthetic(seed=0)
dp = DataPlane(dev, result_shape=(2, B, 5))
pipe = ServingPipeline(se, store, dp, use_graph=True, lookahead=1)
L = N.lib()
e0 = se.engines[0]
nodes = {n.name: n for n in e0.g.nodes}
plans = [p for e in se.engines for p in e.plans]
groups = {"|".join(m.name for m in grp): grp for grp in e0.conv_groups}  # grouped-launch ops by op name


def table(k):
    t = np.zeros((world, DESC_FIELDS), np.int64)
    t[0] = (31, k, 0, (k * B) % store.capacity, B, dp.epoch)
    return t


def recapture():
    torch.cuda.synchronize(dev)
    time.sleep(0.3)  # let the process-group watchdog retire the finished collectives before capturing
    for e in se.engines:
        e.graph_captured = [False] * e.src_slots
    se.capture(pipe.compute_stream)


def ms_per_step() -> float:
    pipe.run(3, table, record=False)
    vals = []
    for _ in range(args.reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        pipe.run(args.steps, table, record=False)
        torch.cuda.synchronize(dev)
        vals.append((time.perf_counter() - t0) / args.steps * 1e3)
    vals.sort()
    return vals[len(vals) // 2]


t_start = time.time()
base = cur = ms_per_step()
print(f"baseline pipeline {base:.4f} ms/step", flush=True)
changes, entries = {}, {}
for i, name in enumerate(e0.op_names):
    if time.time() - t_start > args.budget_s:
        print("time budget reached", flush=True)
        break
    c0 = L.dml_plan_get_cfg(e0.plans[0], i)
    n = nodes.get(name)
    if c0 < 0:
        continue
    if name in groups:  # grouped launch: every other grouped tile, scored in the pipeline only
        grp = groups[name]
        gargs = [e0._conv_args(m) for m in grp if not isinstance(m, Pool)]
        gpools = [e0._pool_args(m) for m in grp if isinstance(m, Pool)]
        key = tuning.group_key(gargs, gpools)
        cands = [c for c in tuning.GROUP_CFGS if c != c0]
    elif isinstance(n, (Conv, Dense, FusedConv)):
        a = e0._conv_args(n)
        key = tuning.shape_key(a)
        alone = []
        for c in tuning.valid_cfgs(a):
            try:
                alone.append((tuning.time_cfg(a, c), c))
            except N.NativeError:
                pass
        alone.sort()
        cands = [c for _, c in alone if c != c0][: args.cands]
    else:
        continue
    best = (cur, c0)
    for c in cands:
        if any(L.dml_plan_set_cfg(p, i, c) < 0 for p in plans):
            continue
        recapture()
        t = ms_per_step()
        if t < best[0]:
            best = (t, c)
    keep = best[0] < cur * (1 - args.thresh)
    print(f"[{i}/{len(e0.op_names)}] {name}: {len(cands)} candidates, best {best[1]} {best[0]:.4f} ms/step "
          f"(current {cur:.4f}, {time.time() - t_start:.0f} s)", flush=True)  # progress (keeps the run visibly alive)
    for p in plans:
        L.dml_plan_set_cfg(p, i, best[1] if keep else c0)
    recapture()
    if keep:
        changes[name] = best[1]
        entries[key] = best[1]
        print(f"{name}: cfg {c0} -> {best[1]}  {cur:.4f} -> {best[0]:.4f} ms/step", flush=True)
        cur = best[0]
final = ms_per_step()
res = {"model": model, "batch": B, "baseline_ms_per_step": round(base, 4), "final_ms_per_step": round(final, 4),
       "changes": changes, "table": entries}
print(json.dumps(res), flush=True)
if args.out:
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
import torch.distributed as dist  # noqa: E402

dist.destroy_process_group()
