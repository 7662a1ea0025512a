"""Sub-batch scheduling experiment: two half-batch engines on two streams,
aligned vs staggered by half a network (so one sub-batch's memory-heavy early
stages overlap the other's compute-heavy late stages).

  python tools/stagger.py --model ResNet50 --batch 256 [--split-frac 0.5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_machine_learning_amd.models import build_model
from distributed_machine_learning_amd.models.engine import Engine

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="ResNet50")
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--split-frac", type=float, default=0.5)
ap.add_argument("--out", default="")
a = ap.parse_args()
g, w = build_model(a.model, seed=0, calibrate=False)
sub = a.batch // 2
A = Engine(g, w, batch=sub)
B = Engine(g, w, batch=sub, share=A)
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
times = A.time_ops(s0)
torch.cuda.synchronize()
tot = sum(t for _, t in times)
acc, mid = 0.0, len(times) // 2
for i, (_, t) in enumerate(times):
    acc += t
    if acc >= a.split_frac * tot:
        mid = i + 1
        break
n = len(times)
for e, s in ((A, s0), (B, s1)):
    e.run(s, use_graph=True)
    e.capture_parts([0, mid, n], s)
torch.cuda.synchronize()


def timeit(fn):
    fn(3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(a.iters)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / a.iters * 1e3


def aligned_free(k):
    for _ in range(k):
        A.run(s0, use_graph=True)
        B.run(s1, use_graph=True)


ev = [torch.cuda.Event() for _ in range(4)]


def aligned_join(k):
    for _ in range(k):
        ev[0].record(s0)
        s1.wait_event(ev[0])
        A.run(s0, use_graph=True)
        B.run(s1, use_graph=True)
        ev[1].record(s1)
        s0.wait_event(ev[1])


def stagger_free(k):
    for _ in range(k):
        A.run_part(0, s0)
        ev[2].record(s0)
        A.run_part(1, s0)
        s1.wait_event(ev[2])
        B.run_part(0, s1)
        B.run_part(1, s1)


def stagger_join(k):
    for _ in range(k):
        ev[0].record(s0)
        A.run_part(0, s0)
        ev[2].record(s0)
        A.run_part(1, s0)
        s1.wait_event(ev[2])
        B.run_part(0, s1)
        B.run_part(1, s1)
        ev[1].record(s1)
        s0.wait_event(ev[1])


res = {"model": a.model, "batch": a.batch, "split_op": mid, "n_ops": n, "split_frac_time": a.split_frac}
for name, fn in (("aligned_free", aligned_free), ("aligned_join", aligned_join), ("stagger_free", stagger_free),
                 ("stagger_join", stagger_join)):
    ms = timeit(fn)
    res[name] = {"ms_per_batch": round(ms, 3), "images_per_s": round(a.batch / ms * 1e3, 1)}
    print(f"{name:14s} {ms:.3f} ms / {a.batch} = {a.batch / ms * 1e3:.0f} img/s", flush=True)
if a.out:
    json.dump(res, open(a.out, "w"), indent=1)
