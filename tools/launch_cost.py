"""Host-side cost of launching one sub-batch forward: hipGraph replay vs the plan's
direct kernel launches (C++ loop of hipLaunchKernelGGL). Prints host enqueue
time (call returns) and GPU completion time for each mode.

  python tools/launch_cost.py [--model ResNet50] [--batch 128] [--iters 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_machine_learning_amd.models import build_model  # noqa: E402
from distributed_machine_learning_amd.models.engine import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="ResNet50")
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()

g, w = build_model(args.model, seed=0, calibrate=False)
eng = Engine(g, w, batch=args.batch)
s = torch.cuda.Stream()
res = {"model": args.model, "batch": args.batch, "ops": len(eng.op_names)}
for mode in ("graph", "direct"):
    ug = mode == "graph"
    eng.run(s, use_graph=ug)
    s.synchronize()
    enq, tot = [], []
    for _ in range(args.iters):
        t0 = time.perf_counter()
        eng.run(s, use_graph=ug)
        t1 = time.perf_counter()
        s.synchronize()
        t2 = time.perf_counter()
        enq.append(t1 - t0)
        tot.append(t2 - t0)
    enq.sort()
    tot.sort()
    res[mode] = {"enqueue_ms_median": round(enq[len(enq) // 2] * 1e3, 3),
                 "total_ms_median": round(tot[len(tot) // 2] * 1e3, 3)}
    # back-to-back launches without syncing: host enqueue rate vs GPU rate
    t0 = time.perf_counter()
    for _ in range(args.iters):
        eng.run(s, use_graph=ug)
    t1 = time.perf_counter()
    s.synchronize()
    t2 = time.perf_counter()
    res[mode]["pipelined_enqueue_ms_per_fwd"] = round((t1 - t0) / args.iters * 1e3, 3)
    res[mode]["pipelined_total_ms_per_fwd"] = round((t2 - t0) / args.iters * 1e3, 3)
print(json.dumps(res))
