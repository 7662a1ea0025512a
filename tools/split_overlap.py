"""How well do the two sub-batch streams of a SplitEngine overlap?

For each launch mode (hipGraph / direct plan launches) and order (extra stream
first / main stream first) it times, with HIP events, the fork -> end of each
sub-batch forward, and the whole split forward; plus the single-engine b/2 and
b forwards for reference. Prints one JSON line.

  python tools/split_overlap.py [--model ResNet50] [--batch 256] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_machine_learning_amd.models import build_model  # noqa: E402
from distributed_machine_learning_amd.models.engine import Engine, SplitEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="ResNet50")
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--iters", type=int, default=10)
args = ap.parse_args()

g, w = build_model(args.model, seed=0, calibrate=False)
se = SplitEngine(g, w, batch=args.batch, splits=2)
main = torch.cuda.Stream()
extra = se.streams[0]
ea, eb = se.engines
res = {"model": args.model, "batch": args.batch}


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record(main)
    for _ in range(iters):
        fn()
    e.record(main)
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for ug in (True, False):
    for order in ("extra_first", "main_first"):
        def fwd(ug=ug, order=order):
            fork = torch.cuda.Event()
            fork.record(main)
            extra.wait_event(fork)
            if order == "extra_first":
                eb.run(extra, use_graph=ug)
                ea.run(main, use_graph=ug)
            else:
                ea.run(main, use_graph=ug)
                eb.run(extra, use_graph=ug)
            j = torch.cuda.Event()
            j.record(extra)
            main.wait_event(j)
        ms = timed(fwd, args.iters)
        # per-stream completion inside one forward
        torch.cuda.synchronize()
        t0, ta, tb = torch.cuda.Event(True), torch.cuda.Event(True), torch.cuda.Event(True)
        t0.record(main)
        extra.wait_event(t0)
        if order == "extra_first":
            eb.run(extra, use_graph=ug)
            ea.run(main, use_graph=ug)
        else:
            ea.run(main, use_graph=ug)
            eb.run(extra, use_graph=ug)
        ta.record(main)
        tb.record(extra)
        torch.cuda.synchronize()
        res[f"{'graph' if ug else 'direct'}_{order}"] = {
            "split_fwd_ms": round(ms, 3), "main_done_ms": round(t0.elapsed_time(ta), 3),
            "extra_done_ms": round(t0.elapsed_time(tb), 3)}
res["single_half_ms"] = round(timed(lambda: ea.run(main, use_graph=True), args.iters), 3)
full = Engine(g, w, batch=args.batch)
res["single_full_ms"] = round(timed(lambda: full.run(main, use_graph=True), args.iters), 3)
print(json.dumps(res))
