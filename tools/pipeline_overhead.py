"""Serving-pipeline overhead at world 1: ms per 256-image ResNet50 batch for
(a) back-to-back SplitEngine forwards (graph replays, alternating source slots,
no staging / collectives) vs (b) the full ServingPipeline (RCCL dispatch,
pinned H2D staging, forward, RCCL gather, host result copy). (b) - (a) is what
the pipeline costs beyond compute. No profiler attached (rocprofv3 serialises
kernels, which hides the two sub-batch streams' overlap).

python tools/pipeline_overhead.py [--model ResNet50] [--steps 40]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributed_machine_learning_amd.models import build_model  # noqa: E402
from distributed_machine_learning_amd.models.engine import SplitEngine  # noqa: E402
from distributed_machine_learning_amd.parallel.dataplane import DESC_FIELDS, DataPlane, init_process_group  # noqa
from distributed_machine_learning_amd.parallel.pipeline import ServingPipeline  # noqa: E402
from distributed_machine_learning_amd.parallel.staging import PinnedImageStore  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="ResNet50")
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--steps", type=int, default=40)
a = ap.parse_args()
rank, world, local = init_process_group()
dev = torch.device("cuda", local)
g, w = build_model(a.model, seed=0)
B = a.batch
eng = SplitEngine(g, w, batch=B, device=str(dev), src_slots=2, splits=2)
s = torch.cuda.Stream(dev)
for k in range(4):
    eng.run(s, use_graph=True, slot=k % 2)
s.synchronize()
t0 = time.perf_counter()
for k in range(a.steps):
    eng.run(s, use_graph=True, slot=k % 2)
s.synchronize()
engine_ms = (time.perf_counter() - t0) / a.steps * 1e3

store = PinnedImageStore(capacity=4 * B, hw=g.input_hw)
store.fill_synthetic(seed=0)
dp = DataPlane(dev, result_shape=(2, B, 5))
pipe = ServingPipeline(eng, store, dp, use_graph=True)


def table(k):
    t = np.zeros((world, DESC_FIELDS), np.int64)
    t[0] = (31, k, 0, (k * B) % store.capacity, B, 0)
    return t


pipe.run(4, table, record=False)
torch.cuda.synchronize()
t0 = time.perf_counter()
st = pipe.run(a.steps, table, record=True)
torch.cuda.synchronize()
pipe_ms = (time.perf_counter() - t0) / a.steps * 1e3
print(json.dumps({"model": a.model, "batch": B, "engine_only_ms": round(engine_ms, 3),
                  "pipeline_ms": round(pipe_ms, 3), "overhead_pct": round(100 * (pipe_ms / engine_ms - 1), 2),
                  "host_wait_s": {k: round(v, 4) for k, v in st.wait_s.items()}}), flush=True)
