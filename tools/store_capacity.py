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


def _profile_threads() -> None:
    """DML_PROFILE_THREADS=<rank>: cProfile the rank's control-plane event loop and its output
    writer thread (each in its own thread), printed when the thread ends."""
    import cProfile
    import pstats

    from distributed_machine_learning_amd.parallel import rank_control, service

    def wrap(fn, label):
        def run(self, *a, **k):
            prof = cProfile.Profile()
            prof.enable()
            try:
                return fn(self, *a, **k)
            finally:
                prof.disable()
                print(f"===== {label}", file=sys.stderr)
                pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(25)
        return run
    rank_control.RankControl._main = wrap(rank_control.RankControl._main, "control loop")
    service.OutputWriter._loop = wrap(service.OutputWriter._loop, "output writer")


class _ThreadCpu:
    """CPU seconds of every thread of this process (/proc/self/task/*/stat utime + stime),
    snapshotted every 0.2 s (threads end before the run returns), named by the Python thread
    that owns it (others: gloo / native pools)."""

    def __init__(self):
        import threading

        self.last, self.names, self.stop = {}, {}, threading.Event()
        self.hz = os.sysconf("SC_CLK_TCK")
        self.t = threading.Thread(target=self._run, daemon=True, name="cpu-snap")
        self.t.start()

    def _snap(self):
        import threading

        for t in threading.enumerate():
            if t.native_id is not None:
                self.names[t.native_id] = t.name.split(" ")[0].rstrip("-0123456789")
        for tid in os.listdir("/proc/self/task"):
            try:
                st = open(f"/proc/self/task/{tid}/stat").read().rsplit(")", 1)[1].split()
            except OSError:
                continue
            self.last[int(tid)] = (int(st[11]) + int(st[12])) / self.hz

    def _run(self):
        while not self.stop.wait(0.2):
            self._snap()

    def result(self) -> dict:
        self.stop.set()
        self.t.join()
        self._snap()
        out = {}
        for tid, cpu in self.last.items():
            name = self.names.get(tid, "native")
            out[name] = round(out.get(name, 0.0) + cpu, 2)
        return out


class _Sampler:
    """Where every Python thread of a rank is, sampled every 2 ms (DML_SAMPLE_RANK=<rank>):
    the innermost frame and three callers per thread, counted; blocked frames skipped."""

    IDLE = {"wait", "select", "_worker", "get", "_watch", "acquire", "sleep"}

    def __init__(self, dt: float = 0.002):
        import collections
        import threading

        self.counts = collections.Counter()
        self.dt, self.stop = dt, threading.Event()
        self.names = {}
        self.t = threading.Thread(target=self._run, daemon=True, name="sampler")
        self.t.start()

    def _run(self):
        import threading

        me = threading.get_ident()
        while not self.stop.wait(self.dt):
            self.names = {t.ident: t.name for t in threading.enumerate()}
            for tid, f in sys._current_frames().items():
                if tid == me:
                    continue
                if f.f_code.co_name in self.IDLE:
                    continue   # blocked (a wait, a select, an idle pool worker): not CPU
                top = f"{os.path.basename(f.f_code.co_filename)}:{f.f_code.co_name}:{f.f_lineno}"
                chain, up = [], f.f_back
                while up is not None and len(chain) < 3:
                    chain.append(f"{os.path.basename(up.f_code.co_filename)}:{up.f_code.co_name}")
                    up = up.f_back
                name = self.names.get(tid, str(tid)).split("_")[0].rstrip("-0123456789")
                self.counts[(name, top, " <- ".join(chain))] += 1

    def report(self, n: int = 40):
        self.stop.set()
        self.t.join()
        per = {}
        for (name, _, _), c in self.counts.items():
            per[name] = per.get(name, 0) + c
        print("sampled threads:", per, file=sys.stderr)
        for (name, top, caller), c in self.counts.most_common(n):
            print(f"{c:6d} {100.0 * c / per[name]:5.1f}%  {name:14s} {top:48s} <- {caller}", file=sys.stderr)


def _rank(rank, world, rdzv, port, batches, rate, out_json, depth=0):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import torch

    torch.set_num_threads(1)
    from distributed_machine_learning_amd.parallel import service_bench
    from distributed_machine_learning_amd.parallel.rank_backend import PacedRankBackend

    import gc
    gcp = {"t": 0.0, "max": 0.0, "n": 0, "total": 0.0}

    def _gc_cb(phase, info):  # the longest cyclic-GC pause of this rank (it holds the GIL throughout)
        if phase == "start":
            gcp["t"] = time.perf_counter()
        else:
            d = time.perf_counter() - gcp["t"]
            gcp["max"], gcp["n"], gcp["total"] = max(gcp["max"], d), gcp["n"] + 1, gcp["total"] + d
    gc.callbacks.append(_gc_cb)
    if os.environ.get("DML_PROFILE_THREADS") == str(rank):
        _profile_threads()
    sampler = _Sampler() if os.environ.get("DML_SAMPLE_RANK") == str(rank) else None
    tcpu = _ThreadCpu()
    t0, c0 = time.perf_counter(), time.process_time()
    prof = None
    if os.environ.get("DML_PROFILE_RANK") == str(rank):  # cProfile of this rank's serve-loop thread
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    bes = []

    def make_backend():
        bes.append(PacedRankBackend(cap=256, batches_per_s=rate))
        return bes[-1]
    rec = service_bench.run(rank, world, None, rdzv, port, batches * 256 * world, 0,
                            {"ResNet50": 256, "InceptionV3": 128}, None, comm="gloo", data_backend="gloo", depth=depth,
                            make_backend=make_backend)
    be = bes[-1] if bes else None
    if sampler is not None:
        sampler.report()

    if prof is not None:
        import pstats
        prof.disable()
        st = pstats.Stats(prof, stream=sys.stderr)
        st.sort_stats("tottime").print_stats(30)
        st.print_callers("acquire|exchange|_poll")
    threads = tcpu.result()
    with open(f"{out_json}.cpu{rank}", "w") as f:  # this rank's CPU seconds (all its threads), GC pauses
        json.dump({"cpu_s": time.process_time() - c0, "gc_max_ms": gcp["max"] * 1e3, "gc_n": gcp["n"],
                   "gc_total_ms": gcp["total"] * 1e3, "objects": len(gc.get_objects()), "threads": threads,
                   "idle_s": be.idle_s if be else 0.0, "idle_n": be.idle_n if be else 0,
                   "span_s": (be.busy_until - be.first) if be and be.real else 0.0,
                   "launched": be.real if be else 0}, f)
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
    per = [json.load(open(f"{out_json}.cpu{r}")) for r in range(world)]
    cpu = [p["cpu_s"] for p in per]
    nb = rec["batches"]["ResNet50"]
    rec["capacity"] = {"world": world, "paced_batches_per_s_per_rank": rate,
                       "batches_per_s": round(nb / rec["elapsed_s"], 1),
                       "batches_per_s_per_rank": round(nb / rec["elapsed_s"] / world, 1),
                       "output_MB_per_s": round(rec["outputs"]["bytes"] / rec["elapsed_s"] / 1e6, 1),
                       "replica_MB_per_s": round(rec["outputs"]["bytes"] * min(4, world) / rec["elapsed_s"] / 1e6, 1),
                       "bytes_per_output": round(rec["outputs"]["bytes"] / max(1, rec["outputs"]["files_stored"])),
                       "cpu_s_per_rank_incl_build": [round(c, 2) for c in cpu], "host_cpus": os.cpu_count(),
                       "gc_max_pause_ms": round(max(p["gc_max_ms"] for p in per), 1),
                       "gc_pause_total_ms_per_rank": [round(p["gc_total_ms"]) for p in per],
                       "gc_tracked_objects_per_rank": [p["objects"] for p in per],
                       "thread_cpu_s_rank0": per[0]["threads"], "thread_cpu_s_coordinator": per[-1]["threads"],
                       # the paced "GPU": launches, first launch -> last completion, and the gaps it sat
                       # idle between (a rank's host side not feeding it)
                       "backend_launched_per_rank": [p["launched"] for p in per],
                       "backend_span_s_per_rank": [round(p["span_s"], 3) for p in per],
                       "backend_idle_s_per_rank": [round(p["idle_s"], 3) for p in per],
                       "backend_idle_gaps_per_rank": [p["idle_n"] for p in per]}
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rate", type=float, default=370.0)
    ap.add_argument("--batches-per-rank", type=int, default=300)
    ap.add_argument("--depth", type=int, default=0, help="batches in flight per rank (0: service.auto_depth)")
    ap.add_argument("--out", default="")
    ap.add_argument("--min-rate", type=float, default=-1.0,
                    help="exit 1 below this many batches/s (-1: 360 x world on a host with >= 64 CPUs, "
                         "else no rate check); the exactly-once listing is always checked")
    a = ap.parse_args()
    rec = measure(a.world, a.rate, a.batches_per_rank, depth=a.depth)
    print(json.dumps(rec["capacity"]), flush=True)
    print(json.dumps({k: rec[k] for k in ("outputs", "loop_phase_s", "steps", "max_batches_per_step",
                                          "jobs_done", "p50_latency_ms", "control_loop_lag_max_ms",
                                          "serve_loop_cpu_s")}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)
    nb = a.world * a.batches_per_rank
    o = rec["outputs"]
    bad = []
    if not (o["failed"] == 0 and o["in_store"] == nb and o["distinct_batches_in_store"] == nb
            and o["listing_duplicates"] == 0):
        bad.append(f"listing not exactly-once: {nb} batches, outputs {o}")
    floor = a.min_rate if a.min_rate >= 0 else (360.0 * a.world if (os.cpu_count() or 1) >= 64 else 0.0)
    if rec["capacity"]["batches_per_s"] < floor:
        bad.append(f"{rec['capacity']['batches_per_s']} batches/s < {floor}")
    print("CAPACITY " + ("FAIL: " + "; ".join(bad) if bad else f"OK: >= {floor:.0f} batches/s, "
                         f"{nb} outputs listed exactly once"), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
