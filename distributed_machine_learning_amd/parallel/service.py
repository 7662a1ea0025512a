"""Elastic multi-GPU serving: coordinator on rank 0, one worker per GPU, RCCL
data plane, SWIM liveness, fair-share scheduling, failure re-dispatch.

Bulk-synchronous steps (BASELINE configs 4 and 5):

  rank 0 (coordinator)  JobManager queues -> fair-share plan over the alive
                        ranks -> descriptor table [world, 6]
  all ranks             RCCL broadcast of the table (control: 48 B per rank)
  each rank             stage its image range (pinned host -> HBM) and run its
                        assigned model's engine (both models resident in HBM)
  all ranks             RCCL gather of packed top-5 results to rank 0
  rank 0                completes batches (C1/C2 metrics, job completion,
                        output_<job>_<batch>_<host>.json via a writer thread)

A rank that dies is detected by SWIM; pending collectives abort, rank 0
requeues the step's in-flight batches at the FRONT of their queues (at-least-
once, like the reference's requeue, worker.py:1284-1306), survivors re-form
the communicator at epoch+1 and serving continues over fewer workers.
Both models' per-batch times are balanced by per-model batch sizes (C3).
"""
from __future__ import annotations

import logging
import os
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..serving.cost_model import CostModel
from ..serving.jobs import MODELS, Batch, JobManager
from ..serving.metrics import Metrics
from ..serving.output import decode_top5, dumps, output_name
from ..serving.scheduler import plan
from .dataplane import DESC_FIELDS, F_BATCH, F_COUNT, F_EPOCH, F_JOB, F_MODEL, F_START
from .elastic import CollectiveFailure, ElasticGroup

log = logging.getLogger(__name__)
MODEL_IDS = {m: i for i, m in enumerate(MODELS)}
IDLE, STOP = -1, -2


# ------------------------------------------------------------- backends ----
class RankBackend:
    """Runs one batch of images [start, start+count) of `model` on this rank.

    ``launch`` is asynchronous on GPU backends: it enqueues staging + forward and
    returns (result [2, max_batch, 5] int32, completion event or None), so the
    service can gather the previous step's results while this batch computes.
    """

    max_batch: int = 256
    device = torch.device("cpu")

    def launch(self, model: str, start: int, count: int, slot: int):
        raise NotImplementedError

    def run(self, model: str, start: int, count: int) -> torch.Tensor:
        res, ev = self.launch(model, start, count, 0)
        if ev is not None:
            ev.synchronize()
        return res


class FakeRankBackend(RankBackend):
    """Deterministic results, optional per-image delay (CPU tests)."""

    def __init__(self, max_batch: int = 16, delay_per_image: float = 0.0):
        self.max_batch, self.delay = max_batch, delay_per_image

    def launch(self, model, start, count, slot):
        if self.delay:
            time.sleep(self.delay * count)
        out = torch.zeros((2, self.max_batch, 5), dtype=torch.int32)
        i = torch.arange(count, dtype=torch.int32)[:, None] + start
        out[0, :count] = (i * 7 + torch.arange(5, dtype=torch.int32)[None] + MODEL_IDS[model] * 100) % 1000
        out[1, :count] = torch.tensor([0.5, 0.2, 0.1, 0.05, 0.01]).view(torch.int32)
        return out, None


class GpuRankBackend(RankBackend):
    """Native engines for both models resident in this GPU's HBM, fed from
    per-model pinned host image arenas. Two source slots per engine: the H2D
    copy of step k (copy stream) overlaps the forward of step k-1 (compute
    stream); results land in one of two output slots."""

    def __init__(self, device: torch.device, batch_sizes: Dict[str, int], arena_images: int = 512, seed: int = 0,
                 models: Sequence[str] = MODELS, splits: int = 2):
        from ..models import build_model
        from ..models.engine import Engine, SplitEngine
        from .staging import PinnedImageStore

        self.device = device
        self.max_batch = max(batch_sizes.values())
        self.engines, self.stores = {}, {}
        self.stream = torch.cuda.Stream(device)
        self.copy_stream = torch.cuda.Stream(device)
        for m in models:
            g, w = build_model(m, seed=seed, calibrate=True)
            b = batch_sizes[m]
            if splits > 1 and b % splits == 0:
                self.engines[m] = SplitEngine(g, w, batch=b, device=str(device), src_slots=2, splits=splits)
            else:
                self.engines[m] = Engine(g, w, batch=b, device=str(device), src_slots=2)
            st = PinnedImageStore(arena_images, g.input_hw)
            st.fill_synthetic(seed=1000 + MODEL_IDS[m])
            self.stores[m] = st
        self.out = [torch.zeros((2, self.max_batch, 5), dtype=torch.int32, device=device) for _ in range(2)]
        self.ev_copied = torch.cuda.Event()
        self.ev_consumed = {(m, k): torch.cuda.Event() for m in models for k in range(2)}
        self.ev_done = [torch.cuda.Event() for _ in range(2)]

    def launch(self, model, start, count, slot):
        eng = self.engines[model]
        cs, s = self.copy_stream, self.stream
        cs.wait_event(self.ev_consumed[(model, slot)])  # WAR: the forward that last read this source slot
        self.stores[model].h2d(eng.srcs[slot], start, min(count, eng.batch), cs)
        self.ev_copied.record(cs)
        s.wait_event(self.ev_copied)
        out = self.out[slot]
        with torch.cuda.stream(s):
            eng.run(s, use_graph=True, slot=slot)
            self.ev_consumed[(model, slot)].record(s)
            out.zero_()
            out[:, : eng.batch].copy_(eng.results[slot])
            self.ev_done[slot].record(s)
        return out, self.ev_done[slot]


# ---------------------------------------------------------- coordinator ----
@dataclass
class Inflight:
    rank: int
    batch: Batch
    t_dispatch: float


class CollectiveCoordinator:
    """Rank-0 scheduling state (the reference leader's job service). Batches are
    tracked per dispatch step, so with the pipelined service two steps (the one
    computing and the one being gathered) can be in flight."""

    def __init__(self, batch_sizes: Dict[str, int], arena_images: Dict[str, int], out_dir: Optional[str] = None,
                 host_tag: str = "node"):
        self.jobs = JobManager(dict(batch_sizes))
        self.cost = CostModel()
        self.metrics = Metrics()
        self.arena = arena_images
        self.inflight: Dict[int, Dict[int, Inflight]] = {}  # step -> global rank -> batch
        self.step_t0: Dict[int, float] = {}
        self.requeued = 0
        self.steps = 0
        self.out_dir = out_dir
        self.host_tag = host_tag
        self._wq: "queue.Queue" = queue.Queue(maxsize=64)
        self._writer = None
        if out_dir:
            os.makedirs(out_dir, exist_ok=True)
            self._writer = threading.Thread(target=self._write_loop, daemon=True)
            self._writer.start()

    def submit(self, model: str, n_images: int) -> int:
        """Cyclic pick over the (replicated, synthetic) arena; image names are
        arena indices so a batch is a contiguous range (one hipMemcpyAsync)."""
        idx = [str(i % self.arena[model]) for i in range(n_images)]
        return self.jobs.submit_images(model, idx, "client", now=time.monotonic()).job_id

    def idle(self) -> bool:
        return self.jobs.pending() == 0 and not self.jobs.inprogress

    def next_table(self, members: List[int], stop_when_idle: bool = True) -> np.ndarray:
        """Descriptor table of dispatch step ``self.steps`` (then increments it)."""
        t = np.full((len(members), DESC_FIELDS), 0, np.int64)
        t[:, F_MODEL] = IDLE
        if stop_when_idle and self.idle():
            t[:, F_MODEL] = STOP
            return t
        queued = {m: len(self.jobs.queues[m]) for m in MODELS}
        workers = [f"rank{g}" for g in members]
        assigns = plan(queued, workers, {}, workers, self.cost, self.jobs.batch_sizes)
        now = time.monotonic()
        cur: Dict[int, Inflight] = {}
        for a in assigns:
            g = int(a.worker[4:])
            b = self.jobs.pop_next(a.model)
            if b is None:
                continue
            r = members.index(g)
            start = int(b.images[0])
            t[r] = (b.job_id, b.batch_id, MODEL_IDS[b.model], start, len(b.images), 0)
            cur[g] = Inflight(g, b, now)
        self.inflight[self.steps] = cur
        self.step_t0[self.steps] = now
        self.steps += 1
        return t

    def complete(self, members: List[int], gathered: Optional[List[torch.Tensor]], step: Optional[int] = None
                 ) -> None:
        """Results of dispatch step ``step`` (default: the oldest in flight) arrived."""
        if step is None:
            if not self.inflight:
                return
            step = min(self.inflight)
        now = time.monotonic()
        service = now - self.step_t0.pop(step, now)
        for g, inf in self.inflight.pop(step, {}).items():
            b = inf.batch
            self.jobs.complete(b.key, now=now)
            n = len(b.images)
            self.metrics.record(b.model, now - inf.t_dispatch, service, n)
            self.cost.observe(b.model, n, service)
            if self._writer is not None and gathered is not None and g in members:
                res = gathered[members.index(g)].cpu().numpy()
                try:
                    self._wq.put_nowait((b, res[0, :n].copy(), res[1, :n].view(np.float32).copy(), g))
                except queue.Full:
                    pass

    def requeue_inflight(self) -> int:
        """Failure: every batch of every in-flight step goes back to the FRONT
        of its queue (newest step first, so queue order is preserved)."""
        n = 0
        for step in sorted(self.inflight, reverse=True):
            for g, inf in self.inflight[step].items():
                if self.jobs.requeue_front(inf.batch.key) is not None:
                    n += 1
        self.inflight.clear()
        self.step_t0.clear()
        self.requeued += n
        return n

    def _write_loop(self) -> None:
        while True:
            b, idx, p, g = self._wq.get()
            if b is None:
                return
            names = [f"synthetic_{b.model}_{i}.jpeg" for i in b.images]
            doc = decode_top5(names, idx, p)
            path = os.path.join(self.out_dir, output_name(b.job_id, b.batch_id, f"{self.host_tag}-rank{g}"))
            with open(path, "w") as f:
                f.write(dumps(doc))

    def flush(self) -> None:
        if self._writer is not None:
            while not self._wq.empty():
                time.sleep(0.01)


# -------------------------------------------------------------- service ----
class CollectiveService:
    """Lag-1 pipelined serving loop, identical on every rank:

      step k:  broadcast table k -> launch batch k (async on the GPU)
               -> gather the results of step k-1 (done or finishing while batch k
                  computes) -> rank 0 completes step k-1.

    so the coordinator's bookkeeping, the descriptor broadcast and the result
    gather hide under the next batch's forward. Any CollectiveFailure requeues
    both in-flight steps and re-forms the communicator over the survivors."""

    def __init__(self, eg: ElasticGroup, backend: RankBackend, coord: Optional[CollectiveCoordinator] = None,
                 kill_rank: int = -1, kill_at_step: int = -1, on_device: bool = False):
        self.eg, self.be, self.coord = eg, backend, coord
        self.kill_rank, self.kill_at_step = kill_rank, kill_at_step
        self.dev = backend.device if on_device else torch.device("cpu")
        self.steps = 0
        self.rebuilds = 0
        self.pending = None  # (step, result tensor, event) of the step awaiting its gather
        self._idle = torch.zeros((2, self.be.max_batch, 5), dtype=torch.int32, device=self.dev)

    def _bufs(self) -> Optional[List[torch.Tensor]]:
        if self.eg.rank != 0:
            return None
        return [torch.zeros((2, self.be.max_batch, 5), dtype=torch.int32, device=self.dev)
                for _ in range(self.eg.world)]

    def _collect(self) -> None:
        """Gather + complete the pending step (all ranks call this in lockstep)."""
        if self.pending is None:
            return
        k, res, ev = self.pending
        if ev is not None:
            if self.dev.type == "cuda":
                torch.cuda.current_stream(self.dev).wait_event(ev)  # RCCL waits on the GPU, not the host
            else:
                ev.synchronize()
        res = res.to(self.dev)
        bufs = self._bufs()
        self.eg.gather(res, bufs)
        self.pending = None
        if self.eg.rank == 0:
            self.coord.complete(self.eg.members, bufs, step=k)

    def step(self) -> bool:
        eg = self.eg
        desc = torch.zeros((eg.world, DESC_FIELDS), dtype=torch.int64, device=self.dev)
        if eg.rank == 0:
            desc.copy_(torch.from_numpy(self.coord.next_table(eg.members)))
        eg.broadcast(desc, 0)
        row = desc[eg.rank].cpu().numpy()
        if row[F_MODEL] == STOP:
            self._collect()
            return False
        if self.steps == self.kill_at_step and eg.grank == self.kill_rank:
            log.warning("rank %d: injected kill at step %d", eg.grank, self.steps)
            os._exit(17)
        if row[F_MODEL] >= 0:
            launched = self.be.launch(MODELS[int(row[F_MODEL])], int(row[F_START]), int(row[F_COUNT]),
                                      self.steps % 2)
        else:
            launched = (self._idle, None)
        self._collect()  # step k-1, overlapping batch k
        self.pending = (self.steps, launched[0], launched[1])
        self.steps += 1
        return True

    def serve(self, max_steps: int = 10 ** 9) -> int:
        while self.steps < max_steps:
            try:
                if not self.step():
                    break
            except CollectiveFailure as e:
                log.warning("rank %d: collective failed (%s); rebuilding", self.eg.grank, e)
                self.pending = None
                if self.eg.rank == 0 and self.eg.grank == 0:
                    self.coord.requeue_inflight()
                deadline = time.monotonic() + 10
                while not (self.eg.dead & set(self.eg.members)) and time.monotonic() < deadline:
                    time.sleep(0.01)  # let SWIM confirm who died
                self.eg.rebuild(set(self.eg.dead), decide=(self.eg.grank == 0))
                self.rebuilds += 1
        else:
            try:
                self._collect()
            except CollectiveFailure:
                pass
        return self.steps
