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
import tempfile
import time
from typing import Dict, List, Optional, Sequence, Tuple


def _pcts(xs) -> dict:
    import numpy as np

    if not xs:
        return {}
    a = np.asarray(xs) * 1e3
    return {"p50": round(float(np.percentile(a, 50)), 2), "p90": round(float(np.percentile(a, 90)), 2),
            "max": round(float(a.max()), 2), "n": len(xs)}


ENCODED_MAX = 2048


def make_jpegs(n: int, seed: int = 0) -> List[Tuple[str, bytes]]:
    """``n`` distinct JPEGs shaped like the reference's ``testfiles/`` (height 300, width
    169-300, ~12 KB): deterministic structured photos — a base colour, two
    low-frequency gratings and pixel noise — so that decoding costs what a real file costs.
    Past ENCODED_MAX, names i >= 2048 carry the bytes of image i % 2048 (encoding 51,200
    photos would take minutes of setup): every NAME is still fetched and decoded once, which is
    what the distinct-image run measures."""
    if n > ENCODED_MAX:
        base = make_jpegs(ENCODED_MAX, seed)
        return [(f"img{i:06d}.jpeg", base[i % ENCODED_MAX][1]) for i in range(n)]
    import io

    import numpy as np
    from PIL import Image

    g = np.random.default_rng(seed)
    out = []
    yy = np.linspace(0.0, 1.0, 300, dtype=np.float32)[:, None]
    noise = g.normal(0, 6, (300, 900, 3)).astype(np.float32)  # one field, a random window per image
    for i in range(n):
        w = int(g.integers(169, 301))
        xx = np.linspace(0.0, 1.0, w, dtype=np.float32)[None, :]
        base = g.uniform(40, 215, 3).astype(np.float32)
        f1, f2 = g.uniform(1, 6, 2)
        ph = g.uniform(0, 6.28, 2)
        img = np.empty((300, w, 3), np.float32)
        for c in range(3):
            img[..., c] = (base[c] + 35 * np.sin(6.28 * f1 * xx + ph[0] + c) + 30 * np.cos(6.28 * f2 * yy + ph[1] - c))
        x0 = int(g.integers(0, 900 - w))
        img += noise[:, x0:x0 + w]
        buf = io.BytesIO()
        Image.fromarray(np.clip(img, 0, 255).astype(np.uint8)).save(buf, format="JPEG", quality=90)
        out.append((f"img_{i:05d}.jpeg", buf.getvalue()))
    return out


def run(rank: int, world: int, device, rdzv: str, swim_base: int, resnet_images: int, inception_images: int,
        batch_sizes: Dict[str, int], out_dir: Optional[str], kills: Sequence[Tuple[int, int]] = (),
        comm: str = "gloo", depth: int = 0, single_rates: Optional[Dict[str, float]] = None,
        make_backend=None, data_backend: str = "nccl", store_images: int = 0,
        decode_threads: int = 0, time_limit_s: float = 0.0) -> Optional[dict]:
    """One rank of the service run; returns the record (on every surviving rank).
    ``store_images`` > 0: the jobs read REAL store images instead of the seeded synthetic
    arena — that many distinct JPEGs are PUT into the replicated store first (outside the
    timed region) and each job picks cyclically over them (worker.py:196-206), so every
    window of images is fetched from the store, decoded once in the whole job and
    replicated to the ranks' HBM arenas (parallel/image_store.py) on the timed path."""
    import torch
    import torch.distributed as dist

    from ..serving.jobs import MODELS
    from .elastic import ElasticGroup
    from .rank_backend import GpuRankBackend
    from .rank_control import RankControl
    from .service import CollectiveService, OutputWriter, ReplicatedCoordinator, rank_switch_interval

    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")  # aborts are ours (parallel/elastic.py)
    rank_switch_interval()
    cap = max(batch_sizes.values())
    t_build = time.perf_counter()
    from .service import STAGE_DEPTH, auto_depth
    from ..utils import numa

    depth = depth or auto_depth(world)
    # store images: room for every distinct image next to the pinned in-flight and staged batches
    arena = max(4 * cap, store_images + world * (depth + STAGE_DEPTH) * cap) if store_images else 4 * cap
    # DML_DECODE_THREADS: the staging pool's size (A/B)
    decode_threads = decode_threads or int(os.environ.get("DML_DECODE_THREADS", "0")) or numa.host_threads(share=1, cap=32)
    loader = {}   # the store loader exists once the control plane runs (below)
    lazy_loader = lambda names: loader["fn"](names)  # noqa: E731
    if make_backend is not None:  # a factory may take the (lazy) store loader
        import inspect

        backend = make_backend(lazy_loader) if inspect.signature(make_backend).parameters else make_backend()
    else:
        backend = GpuRankBackend(device, batch_sizes, cap=cap, arena_images=arena, n_synth=2 * cap,
                                 loader=lazy_loader, decode_threads=decode_threads)
    eg = ElasticGroup(rank, world, store_path=rdzv, backend=comm, device=device if comm == "nccl" else None,
                      timeout_s=120, data_backend=data_backend, shm_exchange=(comm == "gloo"))
    # the product's control plane (serving/rank_main.py): SWIM + election + the replicated
    # store; every output is PUT into the store (bundled, pipelined) before its batch counts
    store_root = os.path.join(os.environ.get("DML_RDZV_DIR", "/tmp"), os.path.basename(rdzv) + "_store")
    ctl = RankControl(rank, world, swim_base, store_dir=os.path.join(store_root, f"rank{rank}"),
                      replication=min(4, world), on_dead=eg.dead.add, on_alive=eg.joiners.add).start()
    loader["fn"] = ctl.store_loader
    kr, kd = -1, -1   # kills: (rank, batches completed when it dies)
    for r, d in kills:
        if r == rank:
            kr, kd = r, d
    coord = ReplicatedCoordinator(batch_sizes, cap=cap, host_tag="mi355x", depth=depth)
    writer = OutputWriter(os.path.join(out_dir, f"rank{rank}") if out_dir else None,
                          put_many_async=ctl.store_put_many_async, host_tag="mi355x")
    # time_limit_s > 0 (a bench pass that must never take the headline record with it): the
    # serve loop raises past the budget instead of the product's watchdog exiting the process
    svc = CollectiveService(eg, backend, coord, control=ctl, writer=writer, kill_rank=kr, kill_at_done=kd,
                            on_device=(comm == "nccl"), watchdog_s=0 if time_limit_s > 0 else 300)
    put_s = 0.0
    if store_images:
        # the JPEGs go into the replicated store first (not timed): the coordinator PUTs them
        # in bundles, every rank then waits at a barrier before the jobs are submitted
        from ..serving.jobs import pick_images

        if svc.is_coordinator():
            t_put = time.perf_counter()
            files = make_jpegs(store_images, seed=11)
            for i in range(0, len(files), 128):
                ok, bad, err = ctl.call(ctl.node.store.put_many(files[i:i + 128]), timeout=120)
                if bad:
                    raise RuntimeError(f"store PUT of the bench images failed: {err}")
            put_s = time.perf_counter() - t_put
            names = ctl.pin_versions(sorted(n for n, _ in files))
            if resnet_images:
                svc.submit_local("ResNet50", images=pick_images(names, resnet_images))
            if inception_images:
                svc.submit_local("InceptionV3", images=pick_images(names, inception_images))
    elif svc.is_coordinator():
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
        getattr(backend, "reset_stats", lambda: None)()
        build_s = time.perf_counter() - t_build
        svc.freeze_heap()
        eg.barrier()
        t0, c0 = time.perf_counter(), time.thread_time()
        prof = None
        if os.environ.get("DML_PROFILE_SERVE") and store_images:   # cProfile of the serve loop (A/B tool)
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        steps = svc.serve(stop_when_idle=True,   # drains the writer: every output file is on disk
                          deadline=time.monotonic() + time_limit_s if time_limit_s > 0 else None)
        loop_cpu = time.thread_time() - c0       # the serve loop thread's own CPU seconds
        if prof is not None:
            import pstats
            prof.disable()
            with open(os.environ["DML_PROFILE_SERVE"], "w") as f:
                pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(40)
                pstats.Stats(prof, stream=f).sort_stats("cumulative").print_stats(40)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        el = time.perf_counter() - t0
        # the slowest survivor's clock (a gloo all-reduce over the final group)
        t = torch.tensor([el], dtype=torch.float64)
        if eg.backend == "gloo":
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0])
        ar = getattr(backend, "arenas", {})
        served = torch.tensor([svc.served_here, writer.written, writer.failed, writer.bytes,
                               int(ctl.loop_lag_max * 1e6),
                               sum(a.decoded for a in ar.values()), sum(a.replicated for a in ar.values()),
                               sum(a.received for a in ar.values()),
                               sum(a.received * a.hw[0] * a.hw[1] * 3 for a in ar.values()),
                               int(loop_cpu * 1e6)], dtype=torch.int64)
        allsv = [torch.zeros_like(served) for _ in range(eg.world)]
        if eg.backend == "gloo":
            dist.all_gather(allsv, served)
        else:
            allsv = [served]
        if svc.is_coordinator():
            # every batch's output is in the store exactly once (the listing is the store
            # leader's metadata, i.e. this rank's): one name per (job, batch)
            listing = ctl.call(ctl.node.store.ls_all("output_*"), timeout=60)
            pairs = {tuple(nm.split("_")[1:3]) for nm in listing}
            c2 = coord.metrics.c2()
            n = {m: coord.metrics.query_count.get(m, 0) for m in MODELS}
            # get-output both ways: rendered at the coordinator from the rows the
            # ranks gathered to it, against the reference's ls-all + fetch + merge of the files
            go = {"collected_rows": svc.collected_rows, "flushes": svc.collect_flushes, "jobs": {}}
            # (the file merge is Python json: bounded to jobs of at most 400k images)
            for jid in sorted(j for j, jb in coord.jobs.jobs.items() if jb.n_images <= 400_000):
                tg = time.perf_counter()
                data = svc.final_output(jid, writer.host_tag, wait_s=2.0)
                tg = time.perf_counter() - tg
                ts = time.perf_counter()
                path = ctl.call(ctl.node.merge_output_files(jid, os.path.join(tempfile.gettempdir(),
                                                                             f"dml_final_{os.getpid()}_{jid}.json")),
                                timeout=300)
                ts = time.perf_counter() - ts
                same = None
                if data is not None and path:
                    with open(path, "rb") as f:
                        same = f.read() == data
                    os.unlink(path)
                go["jobs"][str(jid)] = {"gathered_render_ms": round(tg * 1e3, 2) if data is not None else None,
                                        "merge_files_ms": round(ts * 1e3, 2), "bytes": len(data) if data else 0,
                                        "identical": same}
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
                            "in_store": len(set(listing)), "distinct_batches_in_store": len(pairs),
                            "listing_duplicates": len(listing) - len(set(listing)),
                            "put_bundles_coordinator": writer.bundles,
                            "put_latency_ms_coordinator": _pcts(ctl.put_lat),
                            "writer_busy_s_coordinator": round(writer.busy_s, 3)},
                "get_output": go,
                "steps": steps, "max_batches_per_step": svc.batches_per_step_max,
                "rebuilds": svc.rebuilds, "preempted_batches": coord.preempted, "requeued_batches": coord.requeued,
                "kill_to_redispatch_s": [round(x, 3) for x in svc.recoveries_s],
                "control_loop_lag_max_ms": {f"rank{g}": round(int(v[4]) / 1e3, 1) for g, v in zip(eg.members, allsv)},
                "serve_loop_cpu_s": {f"rank{g}": round(int(v[9]) / 1e6, 3) for g, v in zip(eg.members, allsv)},
                "kills": [f"{r}:{d}" for r, d in kills], "final_members": eg.members,
                "jobs_done": all(j.done for j in coord.jobs.jobs.values()),
                "loop_phase_s": {k: round(v, 4) for k, v in svc.phase_s.items()},
                "loop_phase_max_ms_coordinator": {k: round(v * 1e3, 2) for k, v in svc.phase_max.items()},
                "comm": comm, "depth": depth, "build_s": round(build_s, 1),
                "data": "synthetic uint8 images (seeded HBM arena), random-init weights",
            }
            if store_images:
                col = lambda i: [int(v[i]) for v in allsv]  # noqa: E731 - per rank, member order
                dec = sum(col(5))
                rec["data"] = (f"{store_images} distinct synthetic JPEGs (300 x 169-300, like testfiles/) in the "
                               "replicated store; jobs pick cyclically over them; random-init weights")
                rec["store_path"] = {
                    "distinct_images": store_images, "put_s_untimed": round(put_s, 2),
                    "decode_threads": decode_threads,
                    # whole job: each image decoded once, by the first rank that runs it
                    "decoded": dec, "decode_rate_img_s": round(dec / el, 1),
                    "decoded_per_rank": col(5),
                    "windows_staged_coordinator": int(sum(a.windows_staged for a in ar.values())),
                    "resident_arrivals_per_rank": col(6),
                    # targeted staging: rows shipped HBM to HBM to a rank that re-used an image
                    # another rank held (no all-gather to every rank)
                    "shipped_images_per_rank": col(7), "shipped_bytes": sum(col(8)),
                    "evictions_coordinator": int(sum(a.evictions for a in ar.values())),
                    "decode_cache_hits_coordinator": int(getattr(backend, "decode_hits", 0)),
                    "gpu_jpeg_decodes_coordinator": int(getattr(backend, "gpu_decodes", 0)),
                    "gpu_plane_reuse_coordinator": int(getattr(backend, "plane_hits", 0)),
                    "decode_pool_s_coordinator": {k: round(v, 3) for k, v in getattr(backend, "load_s", {}).items()},
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


def default_kills(world: int, total_batches: int) -> List[Tuple[int, int]]:
    """BASELINE config 5's two worker kills, mid-job: rank 1 once a quarter of the batches
    completed, rank max(2, world-3) at half (two distinct ranks from world 4 on; never the
    coordinator world-1, nor rank 0, whose launcher parent reports the record)."""
    if world < 4:
        raise ValueError("two kills need world >= 4 (rank 0 reports, the coordinator stays)")
    return [(1, total_batches // 4), (max(2, world - 3), total_batches // 2)]


def run_in_children(rank: int, world: int, local_rank: int, rdzv: str, swim_base: int, resnet_images: int,
                    inception_images: int, batch_sizes: Dict[str, int], kills: Sequence[Tuple[int, int]],
                    timeout_s: float = 900.0, backend: str = "gpu", fake_delay: float = 0.0) -> Optional[dict]:
    """(every launcher rank) run this rank's share of a service pass WITH injected kills in
    a child process: a killed rank ends with status 17, which a torchrun worker must not
    (the launcher would tear the whole job down). Never an exec of this process (it holds
    the GPU): a child interpreter, waited for. Returns the record on rank 0 (its child
    survives: kills never target rank 0)."""
    import subprocess
    import sys

    rec_path = f"{rdzv}_rec_{rank}.json"
    cmd = [sys.executable, "-m", "distributed_machine_learning_amd.parallel.service_bench", "--rank", str(rank),
           "--world", str(world), "--rdzv", rdzv, "--port", str(swim_base), "--resnet", str(resnet_images),
           "--inception", str(inception_images), "--batch-resnet", str(batch_sizes["ResNet50"]),
           "--batch-inception", str(batch_sizes["InceptionV3"]), "--out", rec_path,
           "--kills", ",".join(f"{r}:{s}" for r, s in kills), "--backend", backend,
           "--fake-delay", str(fake_delay)]
    env = dict(os.environ, LOCAL_RANK=str(local_rank))
    env.pop("TORCHELASTIC_RUN_ID", None)
    rc = subprocess.run(cmd, env=env, timeout=timeout_s).returncode
    expected = {0, 17} if any(r == rank for r, _ in kills) else {0}
    if rc not in expected:
        raise RuntimeError(f"service kill pass: rank {rank} child exited {rc}")
    if rank != 0:
        if os.path.exists(rec_path):  # every survivor writes the record; rank 0's parent reports it
            os.remove(rec_path)
        return None
    with open(rec_path) as f:
        rec = json.load(f)
    os.remove(rec_path)
    return rec


def _child_main() -> int:
    """The child of run_in_children (one per launcher rank)."""
    import argparse

    import torch

    ap = argparse.ArgumentParser()
    for k in ("--rank", "--world", "--port", "--resnet", "--inception", "--batch-resnet", "--batch-inception"):
        ap.add_argument(k, type=int, required=True)
    ap.add_argument("--rdzv", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--kills", default="")
    ap.add_argument("--backend", default="gpu", choices=("gpu", "fake"))
    ap.add_argument("--fake-delay", type=float, default=0.0, help="fake backend: seconds per image")
    a = ap.parse_args()
    # the data group stays on gloo in this pass: the bench's images are the seeded synthetic
    # arena (no window moves a byte), and a gloo group aborts at once on a dead peer
    device, make_backend, data_backend = None, None, "gloo"
    if a.backend == "gpu":
        device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(device)
    else:
        from .rank_backend import FakeRankBackend

        make_backend = lambda: FakeRankBackend(cap=max(a.batch_resnet, a.batch_inception),  # noqa: E731
                                               delay_per_image=a.fake_delay)
    rec = run(a.rank, a.world, device, a.rdzv, a.port, a.resnet, a.inception,
              {"ResNet50": a.batch_resnet, "InceptionV3": a.batch_inception}, None,
              kills=parse_kills(a.kills.split(",")), make_backend=make_backend, data_backend=data_backend)
    if rec is not None:
        tmp = a.out + ".tmp"
        with open(tmp, "w") as f:
            json.dump(rec, f)
        os.replace(tmp, a.out)
    return 0


if __name__ == "__main__":
    raise SystemExit(_child_main())


def dumps(rec: dict) -> str:
    return json.dumps(rec)
