"""BASELINE configs 4 and 5 as a measured run of the real serving product:
concurrent ResNet50 + InceptionV3 jobs served by the elastic collective service
(parallel/service.py) on every rank of the job, with the product's control plane
(RankControl: SWIM, election, the replicated store) and OUTPUTS ON: every batch's
output_<job>_<batch>_<host>.json is rendered by the rank that ran it and PUT into
the replicated store (bundled, pipelined) before the batch counts as done —
rank_main's configuration — optionally with injected rank kills.

Used by ``bench.py`` (the ``service`` sub-record of the driver's JSON line) and
``tools/serve_bench.py``. Call it in every rank process after the process has
no default process group (the service builds its own, epoch-versioned one).

Reference: the concurrent two-model split (worker.py:255-495, test.py:133-134)
and the kill re-dispatch (worker.py:1279-1306, membershipList.py:46).
"""
from __future__ import annotations

import json
import os
import shutil
import time
from typing import Dict, List, Optional, Sequence, Tuple


def run(rank: int, world: int, device, rdzv: str, swim_base: int, resnet_images: int, inception_images: int,
        batch_sizes: Dict[str, int], out_dir: Optional[str], kills: Sequence[Tuple[int, int]] = (),
        comm: str = "gloo", depth: int = 16, single_rates: Optional[Dict[str, float]] = None,
        make_backend=None, data_backend: str = "nccl") -> Optional[dict]:
    """One rank of the service run; returns the record (on every surviving rank)."""
    import torch
    import torch.distributed as dist

    from ..serving.jobs import MODELS
    from .elastic import ElasticGroup
    from .rank_backend import GpuRankBackend
    from .rank_control import RankControl
    from .service import CollectiveService, OutputWriter, ReplicatedCoordinator

    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")  # aborts are ours (parallel/elastic.py)
    cap = max(batch_sizes.values())
    t_build = time.perf_counter()
    backend = (make_backend() if make_backend is not None else
               GpuRankBackend(device, batch_sizes, cap=cap, arena_images=4 * cap, n_synth=2 * cap))
    eg = ElasticGroup(rank, world, store_path=rdzv, backend=comm, device=device if comm == "nccl" else None,
                      timeout_s=120, data_backend=data_backend, shm_exchange=(comm == "gloo"))
    # the product's control plane (serving/rank_main.py): SWIM + election + the replicated
    # store; every output is PUT into the store (bundled, pipelined) before its batch counts
    store_root = os.path.join(os.environ.get("DML_RDZV_DIR", "/tmp"), os.path.basename(rdzv) + "_store")
    ctl = RankControl(rank, world, swim_base, store_dir=os.path.join(store_root, f"rank{rank}"),
                      replication=min(4, world), on_dead=eg.dead.add, on_alive=eg.joiners.add).start()
    kr, ks = -1, -1
    for r, s in kills:
        if r == rank:
            kr, ks = r, s
    coord = ReplicatedCoordinator(batch_sizes, cap=cap, host_tag="mi355x", depth=depth)
    writer = OutputWriter(os.path.join(out_dir, f"rank{rank}") if out_dir else None,
                          put_many_async=ctl.store_put_many_async, host_tag="mi355x")
    svc = CollectiveService(eg, backend, coord, control=ctl, writer=writer, kill_rank=kr, kill_at_step=ks,
                            on_device=(comm == "nccl"), watchdog_s=300)
    if svc.is_coordinator():
        if resnet_images:
            svc.submit_local("ResNet50", resnet_images)
        if inception_images:
            svc.submit_local("InceptionV3", inception_images)
    rec = None
    try:
        # warm both engines and both slots (graph replay, clocks) outside the timed region
        for m in MODELS:
            for slot in range(min(backend.slots, 2)):
                ev = backend.launch(m, [f"synthetic:{i}" for i in range(batch_sizes[m])], slot)[1]
                if ev is not None:
                    ev.synchronize()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        build_s = time.perf_counter() - t_build
        eg.barrier()
        t0 = time.perf_counter()
        steps = svc.serve(stop_when_idle=True)   # drains the writer: every output file is on disk
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        el = time.perf_counter() - t0
        # the slowest survivor's clock (a gloo all-reduce over the final group)
        t = torch.tensor([el], dtype=torch.float64)
        if eg.backend == "gloo":
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0])
        served = torch.tensor([svc.served_here, writer.written, writer.failed, writer.bytes], dtype=torch.int64)
        allsv = [torch.zeros_like(served) for _ in range(eg.world)]
        if eg.backend == "gloo":
            dist.all_gather(allsv, served)
        else:
            allsv = [served]
        if svc.is_coordinator():
            c2 = coord.metrics.c2()
            n = {m: coord.metrics.query_count.get(m, 0) for m in MODELS}
            tot = sum(n.values())
            per_rank = {f"rank{g}": int(v[0]) for g, v in zip(eg.members, allsv)}
            rec = {
                "metric": "concurrent ResNet50+InceptionV3 serving, outputs on (images/s, whole job)",
                "value": round(tot / el, 1), "unit": "images/s", "n_gpus": world,
                "images_per_s": {m: round(n[m] / el, 1) for m in MODELS},
                "images": n, "elapsed_s": round(el, 4),
                "p50_latency_ms": {m: round(v["query_latency_p50"] * 1e3, 3) for m, v in c2.items()},
                "p90_latency_ms": {m: round(v["query_latency_p90"] * 1e3, 3) for m, v in c2.items()},
                "p99_latency_ms": {m: round(v["query_latency_p99"] * 1e3, 3) for m, v in c2.items()},
                "batches": {m: v["batches"] for m, v in c2.items()},
                "batch_sizes": dict(batch_sizes),
                "fair_share_splits": [s for _, s in coord.split_log][:16],
                "batches_per_rank": per_rank,
                "outputs": {"files_stored": int(sum(int(v[1]) for v in allsv)),
                            "failed": int(sum(int(v[2]) for v in allsv)),
                            "bytes": int(sum(int(v[3]) for v in allsv)), "dir": out_dir or None,
                            "store": f"replicated store, R = {min(4, world)}, bundled PUTs (put_many)",
                            "put_bundles_coordinator": writer.bundles,
                            "writer_busy_s_coordinator": round(writer.busy_s, 3)},
                "steps": steps, "max_batches_per_step": svc.batches_per_step_max,
                "rebuilds": svc.rebuilds, "preempted_batches": coord.preempted, "requeued_batches": coord.requeued,
                "kills": [f"{r}:{s}" for r, s in kills], "final_members": eg.members,
                "jobs_done": all(j.done for j in coord.jobs.jobs.values()),
                "loop_phase_s": {k: round(v, 4) for k, v in svc.phase_s.items()},
                "comm": comm, "depth": depth, "build_s": round(build_s, 1),
                "data": "synthetic uint8 images (seeded HBM arena), random-init weights",
            }
            if single_rates:
                # the same images served one model after the other at the single-model rates
                serial = sum(n[m] / single_rates[m] for m in MODELS if single_rates.get(m))
                rec["vs_time_weighted_single_model"] = round(serial / el, 3)
        # every rank returns the record (bench.py prints it from rank 0)
        if eg.backend == "gloo" and eg.world > 1:
            box = [rec]
            dist.broadcast_object_list(box, src=eg.group_rank_of(svc.coordinator_rank()))
            rec = box[0]
    finally:
        writer.close()
        ctl.stop()
        eg.close()
        if rank == 0:
            if out_dir:
                shutil.rmtree(out_dir, ignore_errors=True)
            shutil.rmtree(store_root, ignore_errors=True)
    return rec


def agree(rank: int) -> Tuple[str, int]:
    """(every rank, while torch.distributed still has the launcher's group)
    a fresh rendezvous path and SWIM base port chosen by rank 0 (a FileStore
    never deletes its file: a reused path would hand out stale epochs)."""
    import socket

    import torch
    import torch.distributed as dist

    t = torch.zeros(2, dtype=torch.int64)
    if rank == 0:
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        t[0] = int(time.time() * 1e6) % (1 << 40) * 1000 + os.getpid() % 1000
        t[1] = min(port, 64000)
    if dist.is_initialized():
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        tt = t.to(dev)
        dist.broadcast(tt, 0)
        t = tt.cpu()
    path = os.path.join(os.environ.get("DML_RDZV_DIR", "/tmp"), f"dml_rdzv_svc_{int(t[0])}")
    return path, int(t[1])


def parse_kills(specs: List[str]) -> List[Tuple[int, int]]:
    return [tuple(int(x) for x in k.split(":")) for k in specs if k]  # type: ignore[misc]


def dumps(rec: dict) -> str:
    return json.dumps(rec)
