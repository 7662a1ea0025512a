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


class ServingPipeline:
    def __init__(self, engine, store: PinnedImageStore, dp: DataPlane, use_graph: bool = True,
                 on_results: Optional[Callable[[BatchRecord], None]] = None, lookahead: int = 2):
        """``lookahead``: how many steps ahead the dispatch broadcast runs. 2 (the
        default) never makes the host wait for a broadcast; 1 dispatches a batch
        only while the previous forward runs — one batch-time less queueing
        latency per query, the host waits for each (µs-scale) broadcast."""
        assert engine.src_slots >= 2, "engine needs 2 source slots for double buffering"
        if lookahead not in (1, 2):
            raise ValueError("lookahead must be 1 or 2")
        self.eng, self.store, self.dp = engine, store, dp
        self.use_graph = use_graph
        self.lookahead = lookahead
        self.on_results = on_results
        dev = engine.device
        self.copy_stream = torch.cuda.Stream(dev)
        self.compute_stream = torch.cuda.Stream(dev)
        self.ev_copied = [torch.cuda.Event() for _ in range(2)]
        self.ev_consumed = [torch.cuda.Event() for _ in range(2)]
        self.ev_res = [torch.cuda.Event() for _ in range(2)]
        self.ev_gathered = [torch.cuda.Event() for _ in range(2)]  # WAR on the slot's result rows
        # a SplitEngine's extra streams wait on these events only (not on the
        # compute stream), so they never idle behind the previous batch's gather
        self._split_deps = hasattr(engine, "engines")
        B = engine.batch
        self.host_res = [torch.empty((dp.world, 2, B, 5), dtype=torch.int32, pin_memory=True) for _ in range(2)]
        if use_graph and hasattr(engine, "capture"):
            engine.capture(self.compute_stream)  # every graph before the first collective (Engine.capture)
        self.stats = PipelineStats()

    def _stage(self, step: int, row: np.ndarray) -> None:
        slot = step % 2
        cs = self.copy_stream
        cs.wait_event(self.ev_consumed[slot])  # WAR: compute(step-2) finished reading this slot
        count = int(row[F_COUNT])
        with _trace.get_tracer().gpu_span("h2d", cs, lane="copy stream", step=step, images=count):
            self.store.h2d(self.eng.srcs[slot], int(row[F_START]), count, cs)
        self.ev_copied[slot].record(cs)

    def run(self, steps: int, table_fn: Callable[[int], np.ndarray], record: bool = True) -> PipelineStats:
        """Serve `steps` batches; table_fn(k) -> descriptor table (used on rank 0).

        Dispatch runs two steps ahead: while batch k computes, the table of
        step k+2 is broadcast (enqueued, not waited on) and the row of step k+1
        (issued one step earlier, so already complete) is read and staged. The
        host therefore never waits behind the forward it just enqueued and the
        GPU always has the next forward queued."""
        dp, eng = self.dp, self.eng
        tr = _trace.get_tracer()
        is0 = dp.rank == 0
        recs: List[BatchRecord] = []
        handles = {}

        def issue(j):
            recs.append(BatchRecord(j, time.perf_counter()))
            if is0:
                tr.begin_async("batch", j, step=j)
            with tr.span("dispatch", step=j):
                handles[j] = dp.issue_dispatch(table_fn(j) if is0 else None)

        issue(0)
        if steps > 1 and self.lookahead == 2:
            issue(1)
        self._stage(0, dp.wait_dispatch(handles.pop(0)))
        prev: Optional[BatchRecord] = None
        ds = dp.dispatch_stream
        for k in range(steps):
            slot = k % 2
            cs = self.compute_stream
            cs.wait_event(self.ev_copied[slot])
            cs.wait_event(self.ev_gathered[slot])  # WAR: gather of step k-2 read this slot's result rows
            with torch.cuda.stream(cs), tr.gpu_span("forward", cs, lane="compute stream", step=k):
                if self._split_deps:
                    eng.run(cs, use_graph=self.use_graph, slot=slot,
                            deps=[self.ev_copied[slot], self.ev_gathered[slot]])
                else:
                    eng.run(cs, use_graph=self.use_graph, slot=slot)
            self.ev_consumed[slot].record(cs)
            if k + 1 < steps:  # stage the next batch (its row was broadcast one step ago)
                if self.lookahead == 1:
                    issue(k + 1)  # dispatched while forward k runs
                tw = time.perf_counter()
                row = dp.wait_dispatch(handles.pop(k + 1))
                self.stats.wait_s["dispatch"] += time.perf_counter() - tw
                self._stage(k + 1, row)
            if self.lookahead == 2 and k + 2 < steps:
                issue(k + 2)
            # result gather + host copy right behind forward k on the compute
            # stream: work on another stream is starved while the forward's
            # kernels fill every CU (measured r2: a gather on the dispatch stream
            # ran only after the NEXT forward drained, and the host waiting for it
            # left a ~270 us GPU bubble per step); in order here it takes ~10 us
            with torch.cuda.stream(cs), tr.gpu_span("gather", cs, lane="compute stream", step=k):
                bufs = dp.gather(eng.results[slot])
                self.ev_gathered[slot].record(cs)
                if is0:
                    hr = self.host_res[slot]
                    for r, b in enumerate(bufs):
                        hr[r].copy_(b, non_blocking=True)
                    self.ev_res[slot].record(cs)
            if prev is not None:
                self._finish(prev, record)
            prev = recs[k]
        if prev is not None:
            self._finish(prev, record)
        self.compute_stream.synchronize()
        ds.synchronize()
        return self.stats

    def _finish(self, rec: BatchRecord, record: bool) -> None:
        slot = rec.step % 2
        tr = _trace.get_tracer()
        if self.dp.rank == 0:
            tw = time.perf_counter()
            with tr.span("wait results", step=rec.step):
                self.ev_res[slot].synchronize()
            self.stats.wait_s["results"] += time.perf_counter() - tw
            rec.t_done = time.perf_counter()
            tr.end_async("batch", rec.step, latency_ms=(rec.t_done - rec.t_dispatch) * 1e3)
            if record:
                self.stats.latencies_s.append(rec.t_done - rec.t_dispatch)
                self.stats.images += self.dp.world * self.eng.batch
            if self.on_results is not None:
                rec.results = [self.host_res[slot][r].clone() for r in range(self.dp.world)]
                self.on_results(rec)
