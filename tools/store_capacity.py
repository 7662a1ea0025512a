#!/usr/bin/env python3
"""Output-store capacity at the 8-GPU batch rate (VERDICT r4 "next round" 3).

World-N gloo run of the shipped serving product (parallel/service_bench.run: the
collective service, the per-rank control plane, the replicated store with R = 4, every
output rendered by the native renderer and PUT before its batch is reported) with a
PacedRankBackend in place of the GPU: each rank completes ``--rate`` ResNet50 b256
batches/s, so the measured rate is what the HOST side sustains — the control
exchange, rendering ~129 KB of JSON per batch and storing it on R ranks.

  python tools/store_capacity.py [--world 8] [--rate 370] [--batches-per-rank 300] [--out f.json]

Reference: the worker PUTs one output file per batch into SDFS and ACKs afterwards
(worker.py:518-537).
"""
import argparse
import json
import multiprocessing as mp
import os
import socket
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_udp_base(n: int) -> int:
    for _ in range(200):
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.bind(("127.0.0.1", 0))
            base = s.getsockname()[1]
        if base + 4 * n < 65000:
            return base
    raise RuntimeError("no port")


def _rank(rank, world, rdzv, port, batches, rate, out_json, depth=0):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import torch

    torch.set_num_threads(1)
    from distributed_machine_learning_amd.parallel import service_bench
    from distributed_machine_learning_amd.parallel.rank_backend import PacedRankBackend

    t0, c0 = time.perf_counter(), time.process_time()
    rec = service_bench.run(rank, world, None, rdzv, port, batches * 256 * world, 0,
                            {"ResNet50": 256, "InceptionV3": 128}, None, comm="gloo", data_backend="gloo", depth=depth,
                            make_backend=lambda: PacedRankBackend(cap=256, batches_per_s=rate))
    with open(f"{out_json}.cpu{rank}", "w") as f:  # this rank's CPU seconds (all its threads)
        f.write(str(time.process_time() - c0))
    if rank == 0 and rec is not None:
        rec["wall_s_incl_build"] = round(time.perf_counter() - t0, 2)
        with open(out_json, "w") as f:
            json.dump(rec, f)


def measure(world: int = 8, rate: float = 370.0, batches_per_rank: int = 300, tmp: str = "", depth: int = 0) -> dict:
    tmp = tmp or tempfile.mkdtemp(prefix="dml_storecap_")
    os.environ["DML_RDZV_DIR"] = tmp
    rdzv = os.path.join(tmp, "rdzv")
    port = _free_udp_base(world)
    out_json = os.path.join(tmp, "rec.json")
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_rank, args=(r, world, rdzv, port, batches_per_rank, rate, out_json, depth))
          for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(900)
    codes = [p.exitcode for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    if codes != [0] * world:
        raise RuntimeError(f"rank exit codes {codes}")
    rec = json.load(open(out_json))
    cpu = [float(open(f"{out_json}.cpu{r}").read()) for r in range(world)]
    nb = rec["batches"]["ResNet50"]
    rec["capacity"] = {"world": world, "paced_batches_per_s_per_rank": rate,
                       "batches_per_s": round(nb / rec["elapsed_s"], 1),
                       "batches_per_s_per_rank": round(nb / rec["elapsed_s"] / world, 1),
                       "output_MB_per_s": round(rec["outputs"]["bytes"] / rec["elapsed_s"] / 1e6, 1),
                       "replica_MB_per_s": round(rec["outputs"]["bytes"] * min(4, world) / rec["elapsed_s"] / 1e6, 1),
                       "bytes_per_output": round(rec["outputs"]["bytes"] / max(1, rec["outputs"]["files_stored"])),
                       "cpu_s_per_rank_incl_build": [round(c, 2) for c in cpu], "host_cpus": os.cpu_count()}
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rate", type=float, default=370.0)
    ap.add_argument("--batches-per-rank", type=int, default=300)
    ap.add_argument("--depth", type=int, default=0, help="batches in flight per rank (0: service.auto_depth)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rec = measure(a.world, a.rate, a.batches_per_rank, depth=a.depth)
    print(json.dumps(rec["capacity"]), flush=True)
    print(json.dumps({k: rec[k] for k in ("outputs", "loop_phase_s", "steps", "max_batches_per_step",
                                          "jobs_done", "p50_latency_ms")}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
