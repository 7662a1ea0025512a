"""Does splitting the per-worker batch into sub-batches on separate HIP streams
(each its own captured hipGraph) beat one big-batch graph? Times graph replays:

  python tools/stream_overlap.py --model ResNet50 --batch 256 --splits 1,2,4
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
ap.add_argument("--splits", default="1,2,4")
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--out", default="")
a = ap.parse_args()
g, w = build_model(a.model, seed=0, calibrate=False)
res = {}
for k in [int(s) for s in a.splits.split(",")]:
    sub = a.batch // k
    engs = [Engine(g, w, batch=sub) for _ in range(k)]
    streams = [torch.cuda.Stream() for _ in range(k)]
    for e, s in zip(engs, streams):
        e.run(s, use_graph=True)
    torch.cuda.synchronize()
    for _ in range(3):
        for e, s in zip(engs, streams):
            e.run(s, use_graph=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        for e, s in zip(engs, streams):
            e.run(s, use_graph=True)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.iters * 1e3
    res[k] = {"ms_per_batch": round(ms, 3), "images_per_s": round(a.batch / ms * 1e3, 1)}
    print(f"splits={k} sub_batch={sub}: {ms:.3f} ms / {a.batch} images = {a.batch / ms * 1e3:.0f} img/s", flush=True)
    del engs
    torch.cuda.empty_cache()
if a.out:
    json.dump({"model": a.model, "batch": a.batch, "results": res}, open(a.out, "w"), indent=1)
