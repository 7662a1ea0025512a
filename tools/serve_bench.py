#!/usr/bin/env python3
"""BASELINE configs 4 and 5 on GPUs: concurrent ResNet50 + InceptionV3 jobs
served by the elastic collective service (one process per GPU, RCCL data
plane, replicated coordinator, SWIM liveness, fair-share scheduler with
per-model batch sizes = C3), optionally with injected rank kills mid-job.

  torchrun --nproc-per-node N tools/serve_bench.py --resnet-images 20480 --inception-images 10240 \\
      [--kill 3:5 --kill 6:9]          # kill global rank 3 at step 5, rank 6 at step 9
  python tools/serve_bench.py ...      # N = 1

Prints one JSON line (the coordinator = highest surviving rank): total
images/s, per-model images/s, p50/p90 query (batch) latency, steps, rebuilds.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--resnet-images", type=int, default=20480)
    ap.add_argument("--inception-images", type=int, default=10240)
    ap.add_argument("--resnet-batch", type=int, default=256)
    ap.add_argument("--inception-batch", type=int, default=128)
    ap.add_argument("--kill", action="append", default=[], help="rank:step")
    ap.add_argument("--out-dir", default="")
    ap.add_argument("--rdzv", default="", help="FileStore rendezvous path (default /tmp/dml_rdzv_<port>)")
    ap.add_argument("--swim-port", type=int, default=0)
    ap.add_argument("--comm", default="gloo", choices=("nccl", "gloo"),
                    help="backend of the service's control collectives (header, log, packed top-5): host gloo "
                         "by default — RCCL kernels for these few-KB messages queue behind the forward's "
                         "kernels (measured 41.0k vs 61.5k img/s concurrent on 1 GPU, profiles/r2_v3)")
    ap.add_argument("--hw-queues", type=int, default=0, help="GPU_MAX_HW_QUEUES for this process (0: HIP default)")
    a = ap.parse_args()
    if a.hw_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(a.hw_queues)  # before the HIP runtime initialises

    import torch

    from distributed_machine_learning_amd.parallel.elastic import ElasticGroup, default_store_path
    from distributed_machine_learning_amd.parallel.fd_thread import RankFailureDetector
    from distributed_machine_learning_amd.parallel.service import (CollectiveService, GpuRankBackend, OutputWriter,
                                                                   ReplicatedCoordinator)

    grank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    base = int(os.environ.get("MASTER_PORT", 29500))
    rdzv = a.rdzv or default_store_path(f"serve_{base}")
    swim_port = a.swim_port or base + 100
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")  # aborts are ours (parallel/elastic.py)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    bs = {"ResNet50": a.resnet_batch, "InceptionV3": a.inception_batch}
    cap = max(bs.values())
    backend = GpuRankBackend(dev, bs, cap=cap, arena_images=4 * cap, n_synth=2 * cap)
    eg = ElasticGroup(grank, world, store_path=rdzv, backend=a.comm, device=dev if a.comm == "nccl" else None,
                      timeout_s=120, data_backend="nccl")  # bulk (image replication) always over RCCL
    fd = RankFailureDetector(grank, world, swim_port, on_dead=eg.dead.add).start()
    kills = [tuple(int(x) for x in k.split(":")) for k in a.kill]
    kr, ks = (-1, -1)
    for r, s in kills:
        if r == grank:
            kr, ks = r, s
    coord = ReplicatedCoordinator(bs, cap=cap, host_tag="mi355x")
    writer = OutputWriter(a.out_dir) if a.out_dir else None
    svc = CollectiveService(eg, backend, coord, writer=writer, kill_rank=kr, kill_at_step=ks,
                            on_device=(a.comm == "nccl"), watchdog_s=300)
    if svc.is_coordinator():
        if a.resnet_images:
            svc.submit_local("ResNet50", a.resnet_images)
        if a.inception_images:
            svc.submit_local("InceptionV3", a.inception_images)
    try:
        # warm both engines and both source slots (graph capture) outside the timed region
        for m in ("ResNet50", "InceptionV3"):
            for slot in (0, 1):
                backend.launch(m, [f"synthetic:{i}" for i in range(bs[m])], slot)[1].synchronize()
        torch.cuda.synchronize()
        eg.barrier()
        t0 = time.perf_counter()
        steps = svc.serve(stop_when_idle=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if svc.is_coordinator():
            c2 = coord.metrics.c2()
            n_r = coord.metrics.query_count.get("ResNet50", 0)
            n_i = coord.metrics.query_count.get("InceptionV3", 0)
            out = {"metric": "concurrent ResNet50+InceptionV3 serving (images/s, whole job)",
                   "value": round((n_r + n_i) / el, 1), "unit": "images/s", "n_gpus": world,
                   "resnet50_images_per_s": round(n_r / el, 1), "inceptionv3_images_per_s": round(n_i / el, 1),
                   "elapsed_s": round(el, 3), "steps": steps, "rebuilds": svc.rebuilds,
                   "final_members": eg.members, "coordinator": svc.coordinator_rank(),
                   "requeued_batches": coord.requeued, "jobs_done": [j.done for j in coord.jobs.jobs.values()],
                   "p50_latency_ms": {m: round(v["query_latency_p50"] * 1e3, 3) for m, v in c2.items()},
                   "p90_latency_ms": {m: round(v["query_latency_p90"] * 1e3, 3) for m, v in c2.items()},
                   "batch_sizes": bs, "kills": a.kill, "dtype": "bf16", "data": "synthetic",
                   "comm": a.comm, "hw_queues": a.hw_queues,
                   "loop_phase_s": {k: round(v, 4) for k, v in svc.phase_s.items()}}
            print(json.dumps(out), flush=True)
    finally:
        fd.stop()
        eg.close()

if __name__ == "__main__":
    main()
