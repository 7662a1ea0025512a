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
images/s over all workers of the headline model (ResNet50 b256, BASELINE config
2); the same run also measures InceptionV3 b128 (config 3) as the
``models.InceptionV3`` sub-record. Data: synthetic uint8 RGB images of the
model's input size, random-init weights of the exact Keras architecture (no
network here). After the timed steps every rank re-runs its last batch through
``Engine.infer`` and rank 0 checks the pipeline's gathered top-5 against it.

  python bench.py --gpus N --steps K --warmup W [--models ResNet50,InceptionV3]

Timing: per model, --spinup-s seconds of untimed steps (clock ramp), then W untimed warmup
steps, then EXACTLY K timed steps between a barrier + device sync on both sides (max over ranks).

Launch: under torchrun (WORLD_SIZE set) each process is one rank. Without it and
with ``--gpus N > 1`` this process becomes a launcher: it spawns N rank
processes (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* env, 127.0.0.1 rendezvous) before
touching the GPU, relays rank 0's JSON line and exits with the worst rank's
status. ``--dry-run`` replaces the GPU step by the dispatch/gather skeleton on
gloo (CPU test of the launcher and of the rank plumbing).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

# one HIP hardware queue per stream (HIP's default is 4 per process): streams sharing a queue run
# in order, so a multi-millisecond JPEG Huffman launch on a side stream held up the compute
# stream mapped to the same queue (rocprofv3, profiles/r5_store). Set before HIP initialises;
# DML_HW_QUEUES overrides.
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("DML_HW_QUEUES", "16")

# the reference's only per-N rates: the scheduler cost model's predicted query
# rate n * batch / time(batch) at batch 10 (worker.py:316-317, models.py:128-139,
# constants worker.py:57-84; BASELINE.md row "Scheduler-predicted query rate").
REF_BATCH_TIME_S = {"ResNet50": 1 * 10 + 3.5 + 1 + 0.25 * 9, "InceptionV3": 1 * 10 + 5.6 + 2 + 0.325 * 9}
DEFAULT_BATCH = {"ResNet50": 256, "InceptionV3": 128}
METRIC = "queries/sec (images/s, whole job) + p50/p90 query latency"


def ref_rate(model: str, n: int) -> float:
    return n * 10 / REF_BATCH_TIME_S[model]


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=120, help="timed steps (120: >= 100 latency samples for p99)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--spinup-s", type=float, default=float(os.environ.get("DML_BENCH_SPINUP_S", "1.0")),
                    help="seconds of untimed steps BEFORE the W warmup steps: the GPU's clocks ramp during the "
                         "first tens of milliseconds of load (per-step kernel time falls ~5 %% over the first "
                         "steps, rocprofv3 trace in profiles/r6_final); reported as `spinup_s`; 0 = off")
    ap.add_argument("--models", default="ResNet50,InceptionV3",
                    help="comma list; the first is the headline `value`, the rest are sub-records")
    ap.add_argument("--model", default="", help="alias: measure only this model")
    ap.add_argument("--batch", type=int, default=0, help="per-worker batch of the headline model "
                    "(default 256 ResNet50 / 128 InceptionV3)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--splits", type=int, default=2,
                    help="sub-batches of the per-worker batch, each on its own HIP stream (1 = one engine)")
    ap.add_argument("--streams", type=int, default=0,
                    help="concurrent streams for the sub-batches (default = --splits); sub-batch i on stream i %% S")
    ap.add_argument("--no-verify", action="store_true", help="skip the post-run top-5 self-check")
    ap.add_argument("--gather-lag", type=int, default=-1, choices=(-1, 0, 1),
                    help="result gather of batch k after forward k+1 on a comm stream (1) or right behind "
                         "forward k (0); -1 = auto: 1 on several GPUs, 0 on one")
    ap.add_argument("--lookahead", type=int, default=0, choices=(0, 1, 2),
                    help="dispatch broadcast runs this many steps ahead; 0 = auto: 1 on one GPU (a "
                         "batch-time less query latency at equal throughput, measured), 2 on several "
                         "(the RCCL broadcast kernel would wait behind the running forward)")
    ap.add_argument("--op-times", default="", help="write per-op times (ms) of one forward to this JSON file")
    ap.add_argument("--trace", default="", help="Chrome-trace JSON of the timed steps ('{rank}' -> rank id)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: gloo dispatch/gather skeleton only (tests the launcher)")
    ap.add_argument("--no-service", action="store_true",
                    help="skip the `service` sub-record (BASELINE config 4: the elastic serving product, "
                         "concurrent ResNet50 + InceptionV3, outputs on)")
    ap.add_argument("--svc-resnet-images", type=int, default=51200, help="ResNet50 images per GPU (service run)")
    ap.add_argument("--svc-inception-images", type=int, default=25600,
                    help="InceptionV3 images per GPU (service run)")
    ap.add_argument("--svc-store-time-limit", type=float, default=300.0,
                    help="seconds each service pass (synthetic, store-image) may serve before it stops (its "
                         "sub-record then covers what completed; the headline record is printed either way)")
    ap.add_argument("--svc-store-images", type=int, default=2048,
                    help="the `service_store` sub-record: the same concurrent jobs over this many distinct JPEGs "
                         "PUT into the replicated store (fetched, decoded once, staged into HBM on the timed path); "
                         "0 = skip")
    ap.add_argument("--svc-outputs", default="",
                    help="also write the service run's output files to this directory (removed afterwards); "
                         "every output is always PUT into the ranks' replicated store, as serving.main --role rank")
    ap.add_argument("--kill", action="append", default=[],
                    help="rank:batches - a kill of the config-5 pass: the rank exits once that many batches completed "
                         "(default: 2 kills, service_bench.default_kills)")
    ap.add_argument("--kill-pass-timeout", type=float, default=300.0, help="seconds for the config-5 pass")
    ap.add_argument("--kill-pass", default="auto", choices=("auto", "on", "off"),
                    help="BASELINE config 5: a second service pass with injected rank kills, run in child "
                         "processes (a killed rank exits 17); auto = on when --gpus >= 4")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher --
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(n: int, argv) -> int:
    """Spawn n rank processes of this script (no GPU call happens here)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))
    out = procs[0].stdout
    for line in iter(out.readline, b""):
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=120))
        except subprocess.TimeoutExpired:
            p.kill()  # exact child pid, never a pattern
            rcs.append(p.wait())
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        print(f"bench launcher: rank exit codes {rcs}", file=sys.stderr)
        return bad[0] if bad[0] > 0 else 1
    return 0


# ------------------------------------------------------------------ per model --
def bench_model(model: str, B: int, args, rank: int, world: int, device, headline: bool) -> dict:
    import numpy as np
    import torch

    from distributed_machine_learning_amd.models import build_model
    from distributed_machine_learning_amd.models.engine import Engine, SplitEngine, merge_point
    from distributed_machine_learning_amd.parallel.dataplane import DESC_FIELDS, DataPlane
    from distributed_machine_learning_amd.parallel.pipeline import ServingPipeline
    from distributed_machine_learning_amd.parallel.staging import PinnedImageStore
    from distributed_machine_learning_amd.utils import trace as _trace

    g, w = build_model(model, seed=0, calibrate=True)
    splits = args.splits if B % max(args.splits, 1) == 0 else 1
    if splits > 1:
        eng = SplitEngine(g, w, batch=B, device=str(device), src_slots=2, splits=splits, streams=args.streams,
                          merge_at=merge_point(model) if splits == 2 else None)
    else:
        eng = Engine(g, w, batch=B, device=str(device), src_slots=2)
    store = PinnedImageStore(capacity=4 * B, hw=g.input_hw)
    store.fill_synthetic(seed=rank)
    dp = DataPlane(device, result_shape=(2, B, 5))
    lookahead = args.lookahead or (1 if world == 1 else 2)
    pipe = ServingPipeline(eng, store, dp, use_graph=not args.no_graph, lookahead=lookahead,
                           gather_lag=None if args.gather_lag < 0 else args.gather_lag)
    cap = store.capacity

    def table(k):
        t = np.zeros((world, DESC_FIELDS), np.int64)
        for r in range(world):
            t[r] = (31, k * world + r, 0, (k * B) % cap, B, dp.epoch)
        return t

    # spin-up (--spinup-s): untimed steps for this many seconds before the warmup, so the timed
    # steps run at the steady clock a serving GPU runs at (20 timed steps at a cold clock measured
    # 47.6k / 90.6-91.1k img/s, 200 steps 50.0k / 93.5-96.0k, 20 after a 1 s spin-up 48.9-49.4k /
    # 93.3-94.6k, InceptionV3 / ResNet50, same box: profiles/r6_final/short_runs.txt)
    # The step count is agreed by every rank (each step runs collectives: a rank-local clock loop
    # would leave the ranks in different collectives): time two steps after a first pair (graph
    # capture), take the slowest rank's, run that many steps.
    if args.spinup_s > 0:
        pipe.run(2, table, record=False)
        torch.cuda.synchronize()
        t_s = time.perf_counter()
        pipe.run(2, table, record=False)
        torch.cuda.synchronize()
        per = dp.max_over_ranks((time.perf_counter() - t_s) / 2)
        pipe.run(max(1, int(min(4000, args.spinup_s / max(per, 1e-4)))), table, record=False)
        torch.cuda.synchronize()
    # warmup (graph capture, clocks, caches)
    pipe.run(max(args.warmup, 1), table, record=False)
    pipe.stats.latencies_s.clear()
    pipe.stats.images = 0
    if args.trace and headline:
        _trace.set_tracer(_trace.Tracer(process_name=f"bench rank {rank}", pid=rank))

    dp.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = pipe.run(args.steps, table, record=True)
    torch.cuda.synchronize()
    dp.barrier()
    elapsed = dp.max_over_ranks(time.perf_counter() - t0)

    verified = None
    if not args.no_verify:
        # the last timed step's gathered rows vs a fresh Engine.infer of the same images
        last = args.steps - 1
        got = pipe.results_of(last).clone() if rank == 0 else None
        start = (last * B) % cap
        idx = [(start + i) % cap for i in range(B)]
        ti, tp = eng.infer(torch.from_numpy(store.array[idx]).to(device))
        expect = torch.stack([ti.to(torch.int32), tp.contiguous().view(torch.int32)])
        torch.cuda.synchronize()
        bufs = dp.gather(expect.contiguous())
        if rank == 0:
            exp = torch.stack([b.cpu() for b in bufs])
            verified = bool(torch.equal(exp, got))
            if not verified:
                bad_ids = (exp[:, 0] != got[:, 0]).sum().item()
                print(f"bench: {model} pipeline top-5 differs from Engine.infer ({bad_ids} ids)", file=sys.stderr)

    if args.trace and headline:
        tr = _trace.get_tracer()
        tr.add_gpu_ops(eng.time_ops(torch.cuda.current_stream()), lane="one sub-batch forward, per op")
        tr.export_chrome(args.trace.replace("{rank}", str(rank)))
        _trace.set_tracer(_trace.Tracer(enabled=False))
    if args.op_times and rank == 0:
        times = eng.time_ops(torch.cuda.current_stream())
        path = args.op_times if headline else args.op_times.replace(".json", f"_{model}.json")
        with open(path, "w") as f:
            json.dump({"model": model, "batch": B // max(splits, 1), "ops": times,
                       "cfg": eng.op_cfg, "total_ms": sum(t for _, t in times)}, f, indent=1)

    rec = None
    if rank == 0:
        value = world * B * args.steps / elapsed
        pct = stats.percentiles()
        rec = {
            "value": round(value, 2),
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "vs_baseline": round(value / ref_rate(model, world), 1),
            "p50_latency_ms": round(pct.get("p50_ms", 0.0), 3),
            "p90_latency_ms": round(pct.get("p90_ms", 0.0), 3),
            "p99_latency_ms": round(pct.get("p99_ms", 0.0), 3),
            "verified_top5": verified,
            "host_wait_s": {k: round(v, 4) for k, v in stats.wait_s.items()},
            "config": {"model": model, "global_batch": B * world, "seq_len": None,
                       "image_hw": list(g.input_hw), "parallelism": f"dp{world}",
                       "per_worker_batch": B, "graph": not args.no_graph, "stream_splits": splits,
                       "streams": eng.nstreams if splits > 1 else 1, "dispatch_lookahead": pipe.lookahead, "gather_lag": pipe.gather_lag,
                       "merged_tail_from": getattr(eng, "merge_at", None)},
            "baseline": {"source": "BASELINE.md scheduler-predicted query rate (cost model, CS425 VMs, TF CPU)",
                         "value": round(ref_rate(model, world), 3), "unit": "images/s"},
        }
    del pipe, eng, store, dp
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return rec


def bench_dry(model: str, B: int, args, rank: int, world: int) -> dict:
    """The rank plumbing without a GPU: gloo dispatch + gather per step."""
    import numpy as np
    import torch

    from distributed_machine_learning_amd.parallel.dataplane import DESC_FIELDS, DataPlane

    dp = DataPlane(torch.device("cpu"), result_shape=(2, B, 5))
    res = torch.zeros((2, B, 5), dtype=torch.int32)
    table = np.zeros((world, DESC_FIELDS), np.int64)
    for _ in range(args.warmup):
        dp.dispatch(table if rank == 0 else None)
        dp.gather(res)
    dp.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        row = dp.dispatch(table if rank == 0 else None)
        res[0, 0, 0] = int(row[1])
        dp.gather(res)
    dp.barrier()
    elapsed = dp.max_over_ranks(time.perf_counter() - t0)
    if rank:
        return None
    return {"value": round(world * B * args.steps / elapsed, 2), "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "vs_baseline": None, "verified_top5": None,
            "config": {"model": model, "global_batch": B * world, "seq_len": None, "parallelism": f"dp{world}",
                       "per_worker_batch": B}}


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch(args.gpus, argv)

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from distributed_machine_learning_amd.utils import numa

    # NUMA-local placement before any GPU call: this rank's threads (and the pinned arenas
    # they first-touch) on the cores of its GPU's socket (utils/numa.py)
    placement = numa.bind_local_rank(int(os.environ.get("LOCAL_RANK", "0")))
    placement["rank"] = int(os.environ.get("RANK", "0"))

    import torch

    from distributed_machine_learning_amd.models import canonical_name
    from distributed_machine_learning_amd.parallel.dataplane import init_process_group

    models = [canonical_name(m) for m in (args.model or args.models).split(",") if m]
    rank, world, local = init_process_group(backend="gloo" if args.dry_run else None)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    device = None
    if not args.dry_run:
        device = torch.device("cuda", local)
        torch.cuda.set_device(device)

    import torch.distributed as dist

    placements = [placement]
    if dist.is_initialized() and world > 1:
        placements = [None] * world
        dist.all_gather_object(placements, placement)

    recs = {}
    for i, m in enumerate(models):
        B = (args.batch if i == 0 and args.batch else 0) or DEFAULT_BATCH[m]
        if args.dry_run:
            recs[m] = bench_dry(m, B, args, rank, world)
        else:
            recs[m] = bench_model(m, B, args, rank, world, device, headline=(i == 0))

    svc = None
    if not args.dry_run and not args.no_service:
        try:  # the headline line is printed whatever happens in the service passes
            svc = bench_service(args, rank, world, device, recs)
        except Exception as e:  # noqa: BLE001 - reported in the record
            print(f"bench: rank {rank}: service pass failed: {e}", file=sys.stderr, flush=True)
            svc = {"error": str(e)[:500]}

    if rank == 0:
        head = recs[models[0]]
        out = {
            "metric": METRIC,
            "value": head["value"],
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "spinup_s": args.spinup_s,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": head["vs_baseline"],
            "dtype": "bf16",
            "data": ("dry-run: dispatch/gather skeleton only, no compute" if args.dry_run else
                     "synthetic uint8 RGB images, random-init weights (Keras architecture)"),
            "config": head["config"],
        }
        for k in ("p50_latency_ms", "p90_latency_ms", "p99_latency_ms", "verified_top5", "host_wait_s", "baseline"):
            if k in head:
                out[k] = head[k]
        if len(models) > 1:
            out["models"] = {m: recs[m] for m in models[1:]}
        if svc is not None:
            out["service"] = svc
        out["placement"] = placements
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


def bench_service(args, rank: int, world: int, device, recs: dict):
    """BASELINE config 4 (and 5 with --kill): the elastic serving product on
    every rank - concurrent ResNet50 b256 + InceptionV3 b128 jobs, fair-share
    with preemption, one control collective per step, outputs written by the
    ranks (parallel/service_bench.py). Weak scaling: images per GPU fixed."""
    import torch.distributed as dist

    from distributed_machine_learning_amd.parallel import service_bench

    rdzv, port = service_bench.agree(rank)
    kill_pass = args.kill_pass == "on" or (args.kill_pass == "auto" and world >= 4)
    if kill_pass:
        rdzv_k, port_k = service_bench.agree(rank)
    if args.svc_store_images:
        rdzv_s, port_s = service_bench.agree(rank)
    dist.destroy_process_group()  # the service builds its own epoch-versioned groups
    rates = {m: r["value"] for m, r in recs.items() if r and "value" in r}
    out_dir = (os.path.join(args.svc_outputs, os.path.basename(rdzv) + "_outputs") if args.svc_outputs else None)
    rec = service_bench.run(rank, world, device, rdzv, port, args.svc_resnet_images * world,
                            args.svc_inception_images * world, dict(DEFAULT_BATCH), out_dir, single_rates=rates,
                            time_limit_s=args.svc_store_time_limit)
    if args.svc_store_images and rec is not None:
        # the reference's real workload: jobs over store images (worker.py:1361-1386) —
        # fetched from the replicated store, decoded once per job, staged into HBM windows
        try:
            srec = service_bench.run(rank, world, device, rdzv_s, port_s, args.svc_resnet_images * world,
                                     args.svc_inception_images * world, dict(DEFAULT_BATCH), None,
                                     single_rates=rates, store_images=args.svc_store_images,
                                     time_limit_s=args.svc_store_time_limit)
        except Exception as e:  # noqa: BLE001 - reported in the record, never fails the headline
            print(f"bench: rank {rank}: store-image service pass failed: {e}", file=sys.stderr, flush=True)
            srec = {"error": str(e)[:500]}
        if srec is not None:
            if "value" in srec and rec.get("value"):
                srec["vs_synthetic_service"] = round(srec["value"] / rec["value"], 3)
            rec["store_images_pass"] = srec
    if kill_pass:
        # BASELINE config 5: the same concurrent jobs with two ranks killed mid-job (SWIM
        # detects, the survivors rebuild and re-dispatch); each rank's share runs in a child
        nb = sum(-(-n * world // DEFAULT_BATCH[m]) for m, n in (("ResNet50", args.svc_resnet_images),
                                                                 ("InceptionV3", args.svc_inception_images)))
        kills = service_bench.parse_kills(args.kill) or service_bench.default_kills(world, nb)
        try:  # never fails the headline record: a kill-pass failure is reported in it
            krec = service_bench.run_in_children(rank, world, device.index or 0, rdzv_k, port_k,
                                                 args.svc_resnet_images * world, args.svc_inception_images * world,
                                                 dict(DEFAULT_BATCH), kills, timeout_s=args.kill_pass_timeout)
        except Exception as e:  # noqa: BLE001
            print(f"bench: rank {rank}: config-5 kill pass failed: {e}", file=sys.stderr, flush=True)
            krec = {"error": str(e)[:500]}
        if rec is not None and krec is not None:
            if "metric" in krec:
                krec["metric"] = "config 5: " + krec["metric"] + ", 2 ranks killed mid-job"
            rec["kill_pass"] = krec
    return rec


if __name__ == "__main__":
    sys.exit(main())
