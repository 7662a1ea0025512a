#!/usr/bin/env python3
"""Headline benchmark: distributed image-classification serving throughput.

Metric (BASELINE.json): queries/sec + p50/p90 query latency, ResNet50 &
InceptionV3 at 1/2/4/8 workers. One worker process per MI355X; rank 0 also runs
the coordinator. Each step = one batch per worker served end to end:

  rank 0 RCCL-broadcasts the dispatch table (job, batch, image range per worker)
  -> every worker hipMemcpyAsync's its uint8 images from its pinned host store
  -> fused preprocess (nearest resize + caffe/tf normalise) -> full bf16 forward
     on the hand-written gfx950 kernels (one hipGraph) -> softmax + top-5
  -> RCCL gather of the packed top-5 results to rank 0 -> host copy at rank 0.

Weak scaling: the per-worker batch is fixed as N grows. ``value`` = total
images/s over all workers. Data: synthetic uint8 RGB images of the model's input
size, random-init weights of the exact Keras architecture (no network here).

  python bench.py --gpus N --steps K --warmup W [--model ResNet50|InceptionV3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# the reference's only per-N rates: the scheduler cost model's predicted query
# rate n * batch / time(batch) at batch 10 (worker.py:316-317, models.py:128-139,
# constants worker.py:57-84; BASELINE.md row "Scheduler-predicted query rate").
REF_BATCH_TIME_S = {"ResNet50": 1 * 10 + 3.5 + 1 + 0.25 * 9, "InceptionV3": 1 * 10 + 5.6 + 2 + 0.325 * 9}
DEFAULT_BATCH = {"ResNet50": 256, "InceptionV3": 128}


def ref_rate(model: str, n: int) -> float:
    return n * 10 / REF_BATCH_TIME_S[model]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="ResNet50")
    ap.add_argument("--batch", type=int, default=0, help="per-worker batch (default 256 ResNet50 / 128 InceptionV3)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--splits", type=int, default=2,
                    help="sub-batches of the per-worker batch, each on its own HIP stream (1 = one engine)")
    ap.add_argument("--streams", type=int, default=0,
                    help="concurrent streams for the sub-batches (default = --splits); sub-batch i on stream i %% S")
    ap.add_argument("--op-times", default="", help="write per-op times (ms) of one forward to this JSON file")
    ap.add_argument("--trace", default="", help="Chrome-trace JSON of the timed steps ('{rank}' -> rank id)")
    args = ap.parse_args()

    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from distributed_machine_learning_amd.models import build_model, canonical_name
    from distributed_machine_learning_amd.models.engine import Engine, SplitEngine
    from distributed_machine_learning_amd.parallel.dataplane import DESC_FIELDS, DataPlane, init_process_group
    from distributed_machine_learning_amd.parallel.pipeline import ServingPipeline
    from distributed_machine_learning_amd.parallel.staging import PinnedImageStore

    from distributed_machine_learning_amd.utils import trace as _trace

    model = canonical_name(args.model)
    B = args.batch or DEFAULT_BATCH[model]
    rank, world, local = init_process_group()
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    g, w = build_model(model, seed=0, calibrate=True)
    if args.splits > 1:
        eng = SplitEngine(g, w, batch=B, device=str(device), src_slots=2, splits=args.splits, streams=args.streams)
    else:
        eng = Engine(g, w, batch=B, device=str(device), src_slots=2)
    store = PinnedImageStore(capacity=4 * B, hw=g.input_hw)
    store.fill_synthetic(seed=rank)
    dp = DataPlane(device, result_shape=(2, B, 5))
    pipe = ServingPipeline(eng, store, dp, use_graph=not args.no_graph)

    cap = store.capacity

    def table(k):
        import numpy as np

        t = np.zeros((world, DESC_FIELDS), np.int64)
        for r in range(world):
            t[r] = (31, k * world + r, 0, (k * B) % cap, B, dp.epoch)
        return t

    # warmup (graph capture, clocks, caches)
    pipe.run(max(args.warmup, 1), table, record=False)
    pipe.stats.latencies_s.clear()
    pipe.stats.images = 0
    if args.trace:
        _trace.set_tracer(_trace.Tracer(process_name=f"bench rank {rank}", pid=rank))

    dp.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = pipe.run(args.steps, table, record=True)
    torch.cuda.synchronize()
    dp.barrier()
    elapsed = dp.max_over_ranks(time.perf_counter() - t0)

    if args.trace:
        tr = _trace.get_tracer()
        tr.add_gpu_ops(eng.time_ops(torch.cuda.current_stream()), lane="one sub-batch forward, per op")
        tr.export_chrome(args.trace.replace("{rank}", str(rank)))
    if args.op_times and rank == 0:
        times = eng.time_ops(torch.cuda.current_stream())
        with open(args.op_times, "w") as f:
            json.dump({"model": model, "batch": B // max(args.splits, 1), "ops": times,
                       "cfg": eng.op_cfg, "total_ms": sum(t for _, t in times)}, f, indent=1)

    if rank == 0:
        total_images = world * B * args.steps
        value = total_images / elapsed
        pct = stats.percentiles()
        out = {
            "metric": "queries/sec (images/s, whole job) + p50/p90 query latency",
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / ref_rate(model, world), 1),
            "dtype": "bf16",
            "data": "synthetic uint8 RGB images, random-init weights (Keras architecture)",
            "config": {"model": model, "global_batch": B * world, "seq_len": None,
                       "image_hw": list(g.input_hw), "parallelism": f"dp{world}",
                       "per_worker_batch": B, "graph": not args.no_graph, "stream_splits": args.splits,
                       "streams": eng.nstreams if args.splits > 1 else 1},
            "p50_latency_ms": round(pct.get("p50_ms", 0.0), 3),
            "p90_latency_ms": round(pct.get("p90_ms", 0.0), 3),
            "p99_latency_ms": round(pct.get("p99_ms", 0.0), 3),
            "baseline": {"source": "BASELINE.md scheduler-predicted query rate (cost model, CS425 VMs, TF CPU)",
                         "value": round(ref_rate(model, world), 3), "unit": "images/s"},
        }
        print(json.dumps(out), flush=True)
    import torch.distributed as dist

    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
