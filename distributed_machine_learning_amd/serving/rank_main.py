"""The MI355X serving product: one rank process per GPU, launched by one command.

  python -m distributed_machine_learning_amd.serving.main --role rank --gpus 8 \\
      [--backend gpu|cpu|fake|store] [--base-port 8700] [--store-dir ./sdfs] [--out-dir ./outputs] \\
      [--batch-resnet 256 --batch-inception 128] [--comm gloo|nccl]

  # re-start ONE rank of a running job (after it died): it re-joins the group
  python -m distributed_machine_learning_amd.serving.main --role rank --rank 3 --rejoin \\
      --rdzv <path printed by the launcher> --gpus 8 --base-port 8700 ...

Reference: one command per node, ``python3 main.py --hostname=H --port=P``
(main.py:15-27), running the failure detector, SDFS replica, leader duties and
CLI in one process (worker.py:2036-2044). Here the launcher (this process)
spawns N rank processes BEFORE anything touches a GPU (never exec: a child per
rank); each rank runs, on GPU ``rank``:
  * ``RankControl``: SWIM membership + bully election (store leader =
    coordinator = highest rank) + the replicated store (blob plane) + the
    job-service handlers the reference leader served (submit-job, C1, C2, C3, C5);
  * ``GpuRankBackend`` (native engines of both models, HBM image stores) fed by
    the store through ``RankControl.store_loader`` (``cpu``: the fp32 PyTorch
    executor on the host — BASELINE config 1, the reference's CPU worker;
    ``fake`` / ``store``: the CPU stand-ins used by tests);
  * ``ElasticGroup`` (control collective on gloo, image replication on RCCL,
    FileStore rendezvous that no rank hosts) + ``CollectiveService`` (replicated
    coordinator, fair-share with preemption, failure rebuild and rejoin);
  * ``OutputWriter``: output_<job>_<batch>_<host>.json PUT into the store (and
    into ``--out-dir`` if given) by the rank that ran the batch.
The CLI (``--role client --introducer 127.0.0.1:<base-port>``) talks to any rank;
FETCH_INTRODUCER answers with the elected leader.

The launcher prints one line ``rank-service: introducer=<addr> rdzv=<path>`` once
the ranks are up, forwards SIGINT/SIGTERM to them (the coordinator then
broadcasts STOP) and exits with the worst rank's status.
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import socket
import subprocess
import sys
import time

# one HIP hardware queue per stream (HIP's default is 4 per process): streams sharing a queue run
# in order, so a multi-millisecond JPEG Huffman launch on a side stream held up the compute
# stream mapped to the same queue (rocprofv3, profiles/r5_store). Set before HIP initialises;
# DML_HW_QUEUES overrides.
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("DML_HW_QUEUES", "16")

log = logging.getLogger(__name__)


def add_args(ap: argparse.ArgumentParser) -> None:
    g = ap.add_argument_group("rank service (--role rank)")
    g.add_argument("--gpus", type=int, default=1, help="rank processes (one per GPU)")
    g.add_argument("--rank", type=int, default=-1, help="run only this rank (child / rejoin mode)")
    g.add_argument("--rejoin", action="store_true", help="this rank re-joins a running job")
    g.add_argument("--rdzv", default="", help="FileStore rendezvous path (unique per job; default: a fresh one)")
    g.add_argument("--base-port", type=int, default=0, help="UDP control port of rank 0 (rank r: +r)")
    g.add_argument("--out-dir", default="", help="also write every output file here")
    g.add_argument("--batch-resnet", type=int, default=256)
    g.add_argument("--batch-inception", type=int, default=128)
    g.add_argument("--comm", default="gloo", choices=("gloo", "nccl"), help="backend of the control collective")
    g.add_argument("--depth", type=int, default=0,
                   help="batches in flight per rank: 2 on the GPU, the rest queued or awaiting their output PUT "
                        "(0: service.auto_depth: 4 on one GPU, 8 with peers)")
    g.add_argument("--replication", type=int, default=4)
    g.add_argument("--arena-images", type=int, default=0,
                   help="HBM image store slots per model beyond the synthetic ones (0: ranks x (depth + staged) x batch, at least 8192)")
    g.add_argument("--no-preempt", action="store_true")


def _free_udp_base(n: int) -> int:
    """A base port with n free UDP ports above it (and their TCP twins free)."""
    for _ in range(100):
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.bind(("127.0.0.1", 0))
            base = s.getsockname()[1]
        if base + n >= 65000:
            continue
        ok = True
        for p in range(base, base + n):
            try:
                with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
                    s.bind(("127.0.0.1", p))
            except OSError:
                ok = False
                break
        if ok:
            return base
    raise RuntimeError("no free port range")


def launch(a: argparse.Namespace, argv) -> int:
    """Spawn a.gpus rank processes of this entry point (no GPU call here)."""
    base = a.base_port or _free_udp_base(a.gpus)
    rdzv = a.rdzv or os.path.join(os.environ.get("DML_RDZV_DIR", "/tmp"),
                                  f"dml_rdzv_rank_{os.getpid()}_{int(time.time() * 1e6)}")
    if os.path.exists(rdzv):
        os.remove(rdzv)  # a FileStore never deletes its file: never reuse one (stale epochs / admissions)
    from ..parallel.elastic import unlink_stale_segments
    unlink_stale_segments(rdzv)  # shared-memory segments a killed previous run over this path left
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus))
        cmd = [sys.executable, "-m", "distributed_machine_learning_amd.serving.main", *argv,
               "--rank", str(r), "--rdzv", rdzv, "--base-port", str(base)]
        procs.append(subprocess.Popen(cmd, env=env))
    print(f"rank-service: introducer=127.0.0.1:{base} rdzv={rdzv} ranks={[p.pid for p in procs]}", flush=True)

    def forward(sig, _frm):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, forward)
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return (bad[0] if bad[0] > 0 else 1) if bad else 0


def rank_main(a: argparse.Namespace) -> int:
    """One rank (this process = GPU ``rank`` of the job)."""
    grank, world = a.rank, a.gpus
    if "backend" not in getattr(a, "explicit", ()):
        a.backend = "gpu"  # the product default of a rank: its GPU
    logging.basicConfig(level=logging.WARNING, format=f"%(asctime)s rank{grank} %(levelname)s %(name)s: %(message)s")
    from ..utils import numa

    # NUMA-local placement before any GPU call (utils/numa.py): the serve loop, the decode
    # pool, the output writer and the pinned arenas they first-touch on the GPU's socket
    local = grank % max(1, int(os.environ.get("LOCAL_WORLD_SIZE", world)))
    placement = numa.bind_local_rank(local) if a.backend == "gpu" else {"bound": False}
    if placement.get("bound"):
        logging.getLogger(__name__).info("rank %d bound to NUMA node %s cpus %s", grank, placement["numa"],
                                         placement["cpus"])
    decode_threads = numa.host_threads(share=numa.ranks_sharing(local, world)) if placement.get("bound") else 8
    import torch

    from ..parallel.elastic import ElasticGroup
    from ..parallel.rank_backend import FakeRankBackend, GpuRankBackend, HostRankBackend, StoreRankBackend
    from ..parallel.rank_control import RankControl
    from ..parallel.service import CollectiveService, OutputWriter, ReplicatedCoordinator, rank_switch_interval
    from .inference import CpuBackend

    if not a.rdzv or not a.base_port:
        raise SystemExit("a rank needs --rdzv and --base-port (use the launcher: --role rank --gpus N)")
    bs = {"ResNet50": a.batch_resnet, "InceptionV3": a.batch_inception}
    cap = max(bs.values())
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")  # aborts are ours (parallel/elastic.py)
    rank_switch_interval()
    dev = None
    if a.backend == "gpu":
        dev = torch.device("cuda", grank % max(torch.cuda.device_count(), 1))
        torch.cuda.set_device(dev)
    store_dir = os.path.join(a.store_dir, f"rank{grank}")
    # SWIM verdicts may arrive before the group exists (a re-joining rank is
    # admitted only once SWIM has seen it): park them until then
    holder, early_dead, early_alive = {}, set(), set()

    def on_dead(g):
        (holder["eg"].dead if "eg" in holder else early_dead).add(g)

    def on_alive(g):
        (holder["eg"].joiners if "eg" in holder else early_alive).add(g)
    ctl = RankControl(grank, world, a.base_port, store_dir=store_dir, replication=min(a.replication, world),
                      rejoin=a.rejoin, on_dead=on_dead, on_alive=on_alive)
    from ..parallel.service import auto_depth

    depth = a.depth or auto_depth(world)
    # the image windows stage world x STAGE_DEPTH batches ahead of dispatch while
    # world x depth are in flight (pinned): the usable arena (beyond the backend's synthetic
    # images) holds both
    from ..parallel.service import STAGE_DEPTH

    need = world * (depth + STAGE_DEPTH) * cap
    if a.arena_images and a.arena_images < need:
        raise SystemExit(f"--arena-images {a.arena_images} < {need} = ranks x (depth + staged) x batch: "
                         "staged-ahead batches would wait behind pinned in-flight ones")
    arena = a.arena_images or max(8192, need)
    backend = {
        "gpu": lambda: GpuRankBackend(dev, bs, cap=cap, arena_images=arena, loader=ctl.store_loader,
                                      decode_threads=decode_threads),
        "fake": lambda: FakeRankBackend(cap=cap, loader=ctl.store_loader),
        "store": lambda: StoreRankBackend(cap=cap, loader=ctl.store_loader),
        "cpu": lambda: HostRankBackend(CpuBackend(), cap=cap, loader=ctl.store_loader),
    }[a.backend]()
    ctl.start()
    eg = ElasticGroup(grank, world, store_path=a.rdzv, backend=a.comm,
                      device=dev if a.comm == "nccl" else None, timeout_s=120,
                      data_backend="nccl" if a.backend == "gpu" else a.comm, join=a.rejoin,
                      shm_exchange=(a.comm == "gloo"))
    eg.dead |= early_dead
    eg.joiners |= {g for g in early_alive if g not in eg.members}
    holder["eg"] = eg
    coord = ReplicatedCoordinator(bs, cap=cap, host_tag="mi355x", depth=depth, preempt=not a.no_preempt)
    writer = OutputWriter(a.out_dir or None, put_many_async=ctl.store_put_many_async, host_tag="mi355x")
    svc = CollectiveService(eg, backend, coord, control=ctl, writer=writer, on_device=(a.comm == "nccl"),
                            watchdog_s=0.0, rejoined=a.rejoin)
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: svc.stop())
    try:
        svc.serve()
        try:
            eg.barrier()  # replicas keep their store nodes up until everyone stopped
        except Exception:
            pass
    finally:
        writer.close()
        ctl.stop()
        eg.close()
    return 0
