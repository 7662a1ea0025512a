"""The per-GPU serving pipeline: dispatch -> stage -> compute -> gather.

Used by bench.py and by the GPU worker runtime. Three HIP streams per rank:

  copy stream     hipMemcpyAsync of batch k+1 (pinned host arena -> HBM slot)
  compute stream  preprocess + forward + softmax/top-5 of batch k (one hipGraph)
  dispatch stream RCCL broadcast of the descriptor table for batch k+1

so staging and dispatch of the next batch hide under the current batch's
compute, and the coordinator (rank 0) consumes batch k-1's gathered results
while batch k runs. Reference equivalent: worker.py:1361-1386 (sequential scp
download of each image, then a fresh ProcessPoolExecutor + model per batch).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import numpy as np
import torch

from ..utils import trace as _trace
from .dataplane import DataPlane, F_COUNT, F_START
from .staging import PinnedImageStore


@dataclass
class BatchRecord:
    step: int
    t_dispatch: float
    t_done: float = 0.0
    results: Optional[List[torch.Tensor]] = None  # rank 0 only (host copies)


@dataclass
class PipelineStats:
    latencies_s: List[float] = field(default_factory=list)
    images: int = 0
    wait_s: dict = field(default_factory=lambda: {"dispatch": 0.0, "results": 0.0, "loop": 0.0})

    def percentiles(self):
        if not self.latencies_s:
            return {}
        a = np.asarray(self.latencies_s) * 1e3
        return {"p50_ms": float(np.percentile(a, 50)), "p90_ms": float(np.percentile(a, 90)),
                "p99_ms": float(np.percentile(a, 99)), "mean_ms": float(a.mean())}


class _NoStream:
    """CPU stand-in of a HIP stream / event (the pipeline's gloo test path): the work
    runs synchronously, in issue order."""

    def wait_event(self, ev) -> None:
        pass

    def record(self, stream=None) -> None:
        pass

    def synchronize(self) -> None:
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class ServingPipeline:
    RING = 4  # result rows in flight: forward k+RING reuses forward k's send/receive buffers

    def __init__(self, engine, store: PinnedImageStore, dp: DataPlane, use_graph: bool = True,
                 on_results: Optional[Callable[[BatchRecord], None]] = None, lookahead: int = 2,
                 gather_lag: Optional[int] = None):
        """``lookahead``: how many steps ahead the dispatch broadcast runs. 2 (the
        default) never makes the host wait for a broadcast; 1 dispatches a batch
        only while the previous forward runs — one batch-time less queueing
        latency per query, the host waits for each (µs-scale) broadcast.
        ``gather_lag``: 0 = the result gather of batch k right behind forward k on the
        compute stream (one rank: the lowest latency); 1 = the gather of batch k is
        issued after forward k+1, on its own comm stream (default when world > 1):
        forward k+1 never waits for the slowest rank's forward k, so rank skew stops
        turning into a per-step bubble on every rank."""
        assert engine.src_slots >= 2, "engine needs 2 source slots for double buffering"
        if lookahead not in (1, 2):
            raise ValueError("lookahead must be 1 or 2")
        self.eng, self.store, self.dp = engine, store, dp
        self.use_graph = use_graph
        self.lookahead = lookahead
        self.gather_lag = (1 if dp.world > 1 else 0) if gather_lag is None else gather_lag
        if self.gather_lag not in (0, 1):
            raise ValueError("gather_lag must be 0 or 1")
        self.on_results = on_results
        dev = engine.device
        self.cuda = torch.device(dev).type == "cuda"
        mk_stream = (lambda: torch.cuda.Stream(dev)) if self.cuda else _NoStream
        mk_event = torch.cuda.Event if self.cuda else _NoStream
        self.copy_stream = mk_stream()
        self.compute_stream = mk_stream()
        self.comm_stream = mk_stream()
        self.ev_copied = [mk_event() for _ in range(2)]
        self.ev_consumed = [mk_event() for _ in range(2)]
        self.ev_fwd = [mk_event() for _ in range(2)]        # forward of the slot's batch done
        self.ev_res = [mk_event() for _ in range(self.RING)]
        self.ev_gathered = [mk_event() for _ in range(self.RING)]  # WAR on a send ring entry
        # a SplitEngine's extra streams wait on these events only (not on the
        # compute stream), so they never idle behind the previous batch's gather
        self._split_deps = hasattr(engine, "engines")
        B = engine.batch
        pin = self.cuda
        self.host_res = [torch.empty((dp.world, 2, B, 5), dtype=torch.int32, pin_memory=pin)
                         for _ in range(self.RING)]
        # lagged gather: forward k's rows are copied out of the engine's result slot into a
        # send ring entry, so forward k+2 reuses the slot without waiting for gather k
        self.send = ([torch.empty((2, B, 5), dtype=torch.int32, device=dev) for _ in range(self.RING)]
                     if self.gather_lag else [])
        self.order: List[tuple] = []   # (op, step) issue order of the last run (tests)
        if use_graph and self.cuda and hasattr(engine, "capture"):
            engine.capture(self.compute_stream)  # every graph before the first collective (Engine.capture)
        self.stats = PipelineStats()

    def _ctx(self, stream):
        return torch.cuda.stream(stream) if self.cuda else stream

    def _stage(self, step: int, row: np.ndarray) -> None:
        slot = step % 2
        cs = self.copy_stream
        cs.wait_event(self.ev_consumed[slot])  # WAR: compute(step-2) finished reading this slot
        count = int(row[F_COUNT])
        with _trace.get_tracer().gpu_span("h2d", cs, lane="copy stream", step=step, images=count):
            self.store.h2d(self.eng.srcs[slot], int(row[F_START]), count, cs)
        self.ev_copied[slot].record(cs)
        self.order.append(("stage", step))

    def results_of(self, step: int) -> torch.Tensor:
        """(rank 0) the gathered rows [world, 2, B, 5] of ``step`` of the last run, once
        it returned (host copy)."""
        return self.host_res[step % self.RING]

    def _gather(self, k: int) -> None:
        """Result gather of batch k (+ rank 0's host copy): right behind forward k on the
        compute stream (lag 0), or on the comm stream behind forward k's event (lag 1)."""
        dp, tr = self.dp, _trace.get_tracer()
        e = k % self.RING
        if self.gather_lag:
            st = self.comm_stream
            st.wait_event(self.ev_fwd[k % 2])
            src = self.send[e]
        else:
            st, src = self.compute_stream, self.eng.results[k % 2]
        with self._ctx(st), tr.gpu_span("gather", st, lane="comm stream" if self.gather_lag else "compute stream",
                                        step=k):
            bufs = dp.gather(src)
            self.ev_gathered[e].record(st)
            if dp.rank == 0:
                hr = self.host_res[e]
                for r, b in enumerate(bufs):
                    hr[r].copy_(b, non_blocking=self.cuda)
                self.ev_res[e].record(st)
        self.order.append(("gather", k))

    def run(self, steps: int, table_fn: Callable[[int], np.ndarray], record: bool = True) -> PipelineStats:
        """Serve `steps` batches; table_fn(k) -> descriptor table (used on rank 0).

        Dispatch runs two steps ahead: while batch k computes, the table of
        step k+2 is broadcast (enqueued, not waited on) and the row of step k+1
        (issued one step earlier, so already complete) is read and staged. The
        host therefore never waits behind the forward it just enqueued and the
        GPU always has the next forward queued. The result gather of batch k is
        issued right after forward k (lag 0) or after forward k+1 (lag 1); the host
        consumes batch k's rows once the gather after it has been issued, so it never
        waits behind a forward it has not yet queued a successor for."""
        dp, eng = self.dp, self.eng
        tr = _trace.get_tracer()
        is0 = dp.rank == 0
        recs: List[BatchRecord] = []
        handles = {}
        lag = self.gather_lag
        self.order = []

        def issue(j):
            recs.append(BatchRecord(j, time.perf_counter()))
            if is0:
                tr.begin_async("batch", j, step=j)
            with tr.span("dispatch", step=j):
                handles[j] = dp.issue_dispatch(table_fn(j) if is0 else None)
            self.order.append(("dispatch", j))

        issue(0)
        if steps > 1 and self.lookahead == 2:
            issue(1)
        self._stage(0, dp.wait_dispatch(handles.pop(0)))
        done = 0  # batches handed to _finish
        for k in range(steps):
            slot, e = k % 2, k % self.RING
            cs = self.compute_stream
            cs.wait_event(self.ev_copied[slot])
            # WAR on the rows forward k writes: the gather that last read them (lag 0: batch
            # k-2 from the result slot; lag 1: batch k-RING from the send ring entry)
            cs.wait_event(self.ev_gathered[(k - 2) % self.RING] if not lag else self.ev_gathered[e])
            with self._ctx(cs), tr.gpu_span("forward", cs, lane="compute stream", step=k):
                if self._split_deps:
                    eng.run(cs, use_graph=self.use_graph, slot=slot,
                            deps=[self.ev_copied[slot], self.ev_gathered[(k - 2) % self.RING]]
                            if not lag else [self.ev_copied[slot], self.ev_fwd[slot]])  # fwd k-2 + its copy-out
                else:
                    eng.run(cs, use_graph=self.use_graph, slot=slot)
                if lag:
                    self.send[e].copy_(eng.results[slot], non_blocking=self.cuda)
            self.ev_consumed[slot].record(cs)
            self.ev_fwd[slot].record(cs)
            self.order.append(("forward", k))
            if k + 1 < steps:  # stage the next batch (its row was broadcast one step ago)
                if self.lookahead == 1:
                    issue(k + 1)  # dispatched while forward k runs
                tw = time.perf_counter()
                row = dp.wait_dispatch(handles.pop(k + 1))
                self.stats.wait_s["dispatch"] += time.perf_counter() - tw
                self._stage(k + 1, row)
            if self.lookahead == 2 and k + 2 < steps:
                issue(k + 2)
            g = k - lag  # the batch whose gather goes out now
            if g >= 0:
                self._gather(g)
            # batches whose gather was issued at least one iteration ago
            while done < g:
                self._finish(recs[done], record)
                done += 1
        for g in range(steps - lag, steps):
            if g >= 0:
                self._gather(g)
        while done < steps:
            self._finish(recs[done], record)
            done += 1
        self.compute_stream.synchronize()
        self.comm_stream.synchronize()
        if self.cuda:
            dp.dispatch_stream.synchronize()
        return self.stats

    def _finish(self, rec: BatchRecord, record: bool) -> None:
        e = rec.step % self.RING
        tr = _trace.get_tracer()
        self.order.append(("finish", rec.step))
        if self.dp.rank == 0:
            tw = time.perf_counter()
            with tr.span("wait results", step=rec.step):
                self.ev_res[e].synchronize()
            self.stats.wait_s["results"] += time.perf_counter() - tw
            rec.t_done = time.perf_counter()
            tr.end_async("batch", rec.step, latency_ms=(rec.t_done - rec.t_dispatch) * 1e3)
            if record:
                self.stats.latencies_s.append(rec.t_done - rec.t_dispatch)
                self.stats.images += self.dp.world * self.eng.batch
            if self.on_results is not None:
                rec.results = [self.host_res[e][r].clone() for r in range(self.dp.world)]
                self.on_results(rec)
