"""Elastic multi-GPU serving: one process per GPU, a REPLICATED coordinator, one
control collective per step, per-rank output writing, SWIM liveness, the
reference's CLI and store.

Reference: the leader (H1) owns all job state and relays submits/ACKs to one
hard-coded standby (H2) over UDP (worker.py:176-495, 887-1037, 577-614); each
worker downloads its images, runs the batch, PUTs its output file into SDFS and
only then ACKs (worker.py:518-537, 1361-1386, 1573-1585); if H1 and H2 die
nothing can take over (election.py:27). Here every rank holds the whole
coordinator state as a replicated state machine driven by ONE all-gather per
step, so ANY survivor can continue as coordinator:

  step k (every rank, at host speed, independent of GPU progress):
    every rank   contributes a fixed-size record: the batches it FINISHED since
                 its last step (output file already written - the reference's
                 PUT-before-ACK - plus the measured service time) and its answers
                 to revoke requests
    coordinator  additionally: the number of new log bytes (client submits / C3
                 / state records, applied by itself before the collective), the
                 step's dispatch table (up to ``depth`` batches per rank in
                 flight: a rank may receive several batches in one step) and
                 revoke requests (preemption of a rank's not-yet-launched
                 batches when the fair-share split moves it to the other model)
    exchange     of those records: every rank gets all of them (gloo: gather to the
                 coordinator + broadcast, two hops at any world size), plus a
                 broadcast of the log bytes when there are any
    every rank   applies, in this order on every rank: log records -> reports ->
                 revoke answers -> the table; identical queues, in-flight sets,
                 job counters and metrics everywhere
    own work     new batches go to the rank's host queue; a batch is launched
                 whenever one of its GPU slots (2) is free; a finished batch's
                 rows go to the rank's output writer thread (native renderer,
                 csrc/host/output_json.cpp), which writes
                 output_<job>_<batch>_<host>.json (and PUTs it into the store)
                 and hands the batch back for the next step's report.
  No rank ever waits for another rank's compute, a step may move many batches
  (the step rate need not match the batch rate), and the coordinator never
  touches result rows.

  The control record is control-sized (~1.5 KB at world 8), so the collective
  runs on a host (gloo) group by default: issued as RCCL kernels they queue
  behind the forward's kernels (profiles/r2_v3). The ``nccl`` backend stays
  supported. Bulk tensors (decoded images) always go over the data group.

Preemption (reference worker.py:389-408, 442-461): when both models have work,
the fair-share split (serving/scheduler.best_split) assigns each rank a model;
a rank moved to the other model gets that model's batches in its free slots at
once, and its queued batches of the old model are revoked - the rank answers
"revoked" for each one still in its host queue (never launched), and every rank
requeues those at the FRONT of their queue. Launched batches finish.

Failure: SWIM (host UDP) confirms a dead rank -> pending collectives abort
(parallel/elastic.py) -> every survivor requeues all in-flight batches at the
FRONT -> the communicator is rebuilt over the survivors -> the new coordinator
broadcasts its full job state first. Outputs of batches that run twice are
rewritten (at-least-once); every job completes.

Rejoin: a restarted rank announces itself over SWIM; the coordinator admits it
at a step boundary (``members<e+1>`` + ``admit<g>`` in the rendezvous store,
GROW flag in the record); every rank requeues its in-flight batches and moves
to epoch e+1 with it; the pre-growth coordinator keeps the role (a joiner stays
out of it until its replica is in sync) and its state record brings the joiner's
replica up to date.

Images: a job names store images (cyclic pick over the sorted ``*.jpeg``
listing, reference worker.py:176-206), pinned to their latest version at submit
time (``name@v``: a later PUT never changes what a queued job reads), or
synthetic images. They are staged in sliding windows just ahead of dispatch
(parallel/image_store.py): every step, every rank hands the batches in flight and
the next queued ones to its backend, which decodes its share of their new images
off the loop and replicates them with one asynchronous all-gather over the data
group (RCCL over xGMI) into a bounded HBM arena — any job size, no whole-job
replication, no stall of the control step. Epoch changes restart the staging.
"""
from __future__ import annotations

import gc
import json
import logging
import os
import queue
import threading
import time
from collections import OrderedDict, deque
from dataclasses import dataclass
from itertools import islice
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..serving.cost_model import CostModel
from ..serving.jobs import MODELS, Batch, JobManager, as_names, json_default
from ..serving.metrics import Metrics
from ..serving.output import BatchRenderer, output_name
from ..serving.scheduler import best_split
from .elastic import CollectiveFailure, ElasticGroup
from .rank_backend import (MODEL_IDS, SLOTS, SYNTH, FakeRankBackend, GpuRankBackend, HostRankBackend,  # noqa: F401
                           RankBackend, StoreRankBackend, synthetic_names)

log = logging.getLogger(__name__)

# ------------------------------------------------------------- the record ----
# Every rank contributes one int64 record of rec_len(world, depth) words per step.
H_VALID, H_LOGLEN, H_STEP, H_FLAGS, H_NREP, H_NACK, H_NREQ, H_GROW = range(8)
HDR = 8
F_STOP, F_GROW, F_FLUSH = 1, 2, 4   # F_FLUSH: every rank flushes its result rows this step
RP_MAX = 16          # reports per rank per step (more wait for the next step)
RV_MAX = 8           # revoke requests per step / answers per rank per step
REP_W = 4            # report: job, batch, service_us, attempts
ACK_W = 3            # revoke answer: job, batch, revoked
REQ_W = 3            # revoke request: global rank, job, batch
TAB_W = 3            # table entry: job, batch, model id (-1 = empty)


def rec_len(world: int, depth: int) -> int:
    return HDR + world * depth * TAB_W + RV_MAX * REQ_W + RP_MAX * REP_W + RV_MAX * ACK_W


def _offs(world: int, depth: int) -> Tuple[int, int, int, int]:
    tab = HDR
    req = tab + world * depth * TAB_W
    rep = req + RV_MAX * REQ_W
    ack = rep + RP_MAX * REP_W
    return tab, req, rep, ack


# ------------------------------------------------------------- coordinator ----
@dataclass
class Inflight:
    rank: int
    batch: Batch
    t_dispatch: float
    seq: int            # dispatch order (requeue restores queue order)


class ReplicatedCoordinator:
    """The job service's state machine (reference leader, worker.py:176-495,
    989-1037), identical on every rank: log records, reports, revoke answers
    and dispatch tables are applied in the same order everywhere. Only the
    active coordinator PLANS (its cost model is timing-dependent). Each rank
    may hold up to ``depth`` dispatched, unfinished batches."""

    def __init__(self, batch_sizes: Dict[str, int], cap: int = 256, host_tag: str = "node", depth: int = 4,
                 preempt: bool = True, gpu_slots: int = SLOTS):
        self.cap, self.depth, self.preempt, self.gpu_slots = cap, depth, preempt, gpu_slots
        self.jobs = JobManager({m: min(int(b), cap) for m, b in batch_sizes.items()})
        self.cost = CostModel()
        self.metrics = Metrics()
        self.inflight: "OrderedDict[tuple, Inflight]" = OrderedDict()   # batch key -> assignment
        self.revoking: set = set()          # keys with an unanswered revoke request
        self.seq = 0
        self.requeued = 0
        self.preempted = 0
        self.host_tag = host_tag
        self.lock = threading.RLock()      # control-thread readers (C1/C2/C5/status) vs the serve loop
        self.split_log: List[Tuple[float, Dict[str, int]]] = []   # (t, ranks per model) when the split changes
        self._last_split: Dict[str, int] = {}
        self._slice_imgs: Dict[str, int] = dict.fromkeys(MODELS, 0)   # one-rank time slice: images dispatched
        # queued batch -> the rank its images are staged for (image windows, parallel/image_store.py):
        # replicated like the rest (assign_affinity runs at the same point on every rank); the
        # plan dispatches a batch to its affinity rank first
        self.affinity: Dict[str, Dict[tuple, int]] = {m: {} for m in MODELS}
        # C5 history: which rank ran each recent batch and the output file it stored (the
        # reference named the worker in the file name, worker.py:1580; one name per batch here)
        self.history: "deque[dict]" = deque(maxlen=4096)

    # ------------------------------------------------------------- log ----
    def apply(self, rec: dict) -> dict:
        """Apply one replicated log record; returns what the requester is told."""
        op = rec["op"]
        if op == "submit":
            job = self.jobs.submit_images(rec["model"], as_names(rec["images"]), rec.get("requester", "client"),
                                          now=time.monotonic(), job_id=int(rec["job_id"]))
            return {"jobid": job.job_id, "batches": job.batches_total}
        if op == "batch_size":
            bs = max(1, min(int(rec["batch_size"]), self.cap))
            self.jobs.set_batch_size(rec["model"], bs)
            return {"model": rec["model"], "batch_size": bs}
        if op == "state":  # the coordinator's full state after a rebuild / growth
            self.jobs.restore(rec["jobs"], requeue_inprogress=True)
            self.inflight.clear()
            self.revoking.clear()
            self.reset_affinity()
            return {}
        raise ValueError(f"unknown log record {op}")

    def next_job_id(self, pending: int = 0) -> int:
        """Id the next submit will get once applied (records apply in order)."""
        return max([30] + list(self.jobs.jobs)) + 1 + pending

    def idle(self) -> bool:
        return self.jobs.pending() == 0 and not self.jobs.inprogress

    def outstanding(self, grank: int) -> int:
        return sum(1 for inf in self.inflight.values() if inf.rank == grank)

    # ---------------------------------------------------------- affinity ----
    def reset_affinity(self) -> None:
        for a in self.affinity.values():
            a.clear()

    def assign_affinity(self, model: str, queued: Sequence[Batch], members: List[int]) -> Dict[tuple, int]:
        """(every rank, same step, same inputs) give each of these queued batches that has
        none the rank its images will be staged for: among the ranks running ``model`` now
        (their latest dispatched batch), the one with the fewest batches of it in flight or
        assigned; none while no rank runs the model (its first batches are staged when they
        are dispatched). Returns the model's affinity map."""
        aff = self.affinity[model]
        todo = [b for b in queued if b.key not in aff]
        if not todo:
            return aff
        last: Dict[int, str] = {}
        load: Dict[int, int] = {}
        for inf in self.inflight.values():   # dispatch order: the last one per rank wins
            last[inf.rank] = inf.batch.model
            if inf.batch.model == model:
                load[inf.rank] = load.get(inf.rank, 0) + 1
        running = [g for g in members if last.get(g) == model]
        if not running:
            return aff
        load = {g: load.get(g, 0) for g in running}
        for g in aff.values():
            if g in load:
                load[g] += 1
        for b in todo:
            g = min(running, key=lambda r: (load[r], r))
            aff[b.key] = g
            load[g] += 1
        return aff

    # ---------------------------------------------------------- planning ----
    def plan(self, members: List[int]) -> Tuple[Dict[int, List[Batch]], List[Tuple[int, tuple]]]:
        """(active coordinator) This step's dispatches {rank: [batches]} and
        revoke requests [(rank, key)]. One model with work: every rank gets its
        batches. Both: the reference's fair-share split (worker.py:303-324) over
        all ranks; ranks keep their current model while its share allows, and
        a rank moved to the other model has its queued (not launched) batches
        of the old model revoked (worker.py:389-408, 442-461)."""
        queued = {m: len(self.jobs.queues[m]) for m in MODELS}
        if not any(queued.values()) or not members:
            return {}, []
        mine: Dict[int, List[Inflight]] = {g: [] for g in members}
        for inf in self.inflight.values():
            if inf.rank in mine:
                mine[inf.rank].append(inf)
        cur = {g: (mine[g][-1].batch.model if mine[g] else None) for g in members}
        active = [m for m in MODELS if queued[m] > 0]
        target: Dict[int, str] = {}
        if len(active) == 1:
            target = {g: active[0] for g in members}
            self._slice_imgs = dict.fromkeys(MODELS, 0)
        elif len(members) == 1 and ONE_RANK_SLICE:
            # one rank, both models: the reference's split needs two workers (worker.py:303-324
            # gives one worker to one model until its queue drains). The rank is time-sliced
            # instead: each step's free slots go to the model with fewer images dispatched since
            # both were queued, so the two jobs advance together at equal image rates (its two
            # GPU slots may hold one batch of each); no revokes between the two
            g = members[0]
            shared = {"InceptionV3": 1, "ResNet50": 1, "time_sliced": 1}
            if self._last_split != shared:   # entering the slice: counts from here on
                self._last_split = dict(shared)
                self.split_log.append((time.monotonic(), dict(shared)))
                self._slice_imgs = dict.fromkeys(MODELS, 0)
            target = {g: min(active, key=lambda m: (self._slice_imgs.get(m, 0), m))}
        else:
            a, b = "InceptionV3", "ResNet50"
            bs = self.jobs.batch_sizes
            ca, cb = best_split(len(members), self.cost.rate_per_worker(a, bs[a]),
                                self.cost.rate_per_worker(b, bs[b]))
            want = {a: ca, b: cb}
            have = {a: 0, b: 0}
            for g in members:  # ranks keep their model while its share allows (lowest ranks first)
                m = cur[g]
                if m in want and have[m] < want[m]:
                    target[g] = m
                    have[m] += 1
            for g in members:  # idle / excess ranks fill the deficits
                if g not in target:
                    m = a if have[a] < want[a] else b
                    target[g] = m
                    have[m] += 1
            if have != self._last_split:
                self._last_split = dict(have)
                self.split_log.append((time.monotonic(), dict(have)))
        disp: Dict[int, List[Batch]] = {}
        revokes: List[Tuple[int, tuple]] = []
        free: Dict[int, int] = {}
        for g in members:
            m = target[g]
            if self.preempt and len(members) > 1 and cur[g] is not None and cur[g] != m:
                # this rank's batches of the old model beyond its GPU slots are
                # still in its host queue: revoke them
                old = [inf for inf in mine[g] if inf.batch.model != m]
                for inf in old[self.gpu_slots:]:
                    if inf.batch.key not in self.revoking and len(revokes) < RV_MAX:
                        revokes.append((g, inf.batch.key))
            # batches being revoked do not hold a slot: the new model starts at once
            # (a revoke that comes too late - the batch was launched - overfills the
            # rank's queue by at most that batch)
            gone = {k for gg, k in revokes if gg == g} | self.revoking
            free[g] = self.depth - sum(1 for inf in mine[g] if inf.batch.key not in gone)
        # every free slot of this step lies within the first world x depth queued batches. One
        # pass over each model's head sorts them: staged for a rank that takes this model now
        # (its own), or orphans (staged for nobody, or for a rank that left / switched model)
        own: Dict[int, List[Batch]] = {}
        orphans: Dict[str, List[Batch]] = {}
        rest: Dict[str, List[Batch]] = {}
        for m in MODELS:
            if not any(target[g] == m and free[g] > 0 for g in members):
                continue
            aff = self.affinity[m]
            orph = orphans[m] = []
            head = rest[m] = list(islice(self.jobs.queues[m], 0, len(members) * self.depth))
            for b in head:
                g = aff.get(b.key) if aff else None
                if g is not None and target.get(g) == m:
                    own.setdefault(g, []).append(b)
                else:
                    orph.append(b)
        used: set = set()

        def take(g: int, cand: List[Batch], i: int = 0) -> int:
            while free[g] > 0 and i < len(cand):
                b = cand[i]
                i += 1
                if b.key not in used:
                    disp.setdefault(g, []).append(b)   # popped for real by apply_table
                    used.add(b.key)
                    free[g] -= 1
            return i
        # 1. the queued batches whose images are staged for this rank; 2. (queue order) the
        # orphans; 3. a rank that would run dry takes any queued batch (its images are then
        # shipped to it)
        for g in members:
            if free[g] > 0 and g in own:
                take(g, own[g])
        pos = {m: 0 for m in orphans}
        for g in members:
            m = target[g]
            if free[g] > 0 and m in orphans:
                pos[m] = take(g, orphans[m], pos[m])
        low = self.depth - max(self.gpu_slots, self.depth // 4)
        for g in members:
            if free[g] > low and target[g] in rest:
                take(g, rest[target[g]])
        if len(members) == 1 and len(active) == 2:
            for bs in disp.values():
                for b in bs:
                    self._slice_imgs[b.model] = self._slice_imgs.get(b.model, 0) + len(b.images)
        return disp, revokes

    def table(self, members: List[int], disp: Dict[int, List[Batch]]) -> np.ndarray:
        t = np.full((len(members), self.depth, TAB_W), -1, np.int64)
        for g, bl in disp.items():
            r = members.index(g)
            for d, b in enumerate(bl[:self.depth]):
                t[r, d] = (b.job_id, b.batch_id, MODEL_IDS[b.model])
        return t

    def apply_table(self, table: np.ndarray, members: List[int]) -> Dict[int, List[Batch]]:
        """Take exactly the dispatched batches out of the local queues (every
        rank); returns {rank: [batches]}."""
        now = time.monotonic()
        out: Dict[int, List[Batch]] = {}
        for r, g in enumerate(members):
            for d in range(table.shape[1]):
                if int(table[r, d, 2]) < 0:
                    continue
                model = MODELS[int(table[r, d, 2])]
                b = self.jobs.pop_key(model, (int(table[r, d, 0]), int(table[r, d, 1])))
                if b is None:
                    raise RuntimeError(f"replica diverged: batch {table[r, d, 0]}:{table[r, d, 1]} not queued")
                self.affinity[model].pop(b.key, None)   # staged for the rank it now runs on
                self.inflight[b.key] = Inflight(g, b, now, self.seq)
                self.seq += 1
                out.setdefault(g, []).append(b)
        return out

    def apply_requests(self, reqs: List[Tuple[int, tuple]]) -> None:
        for _, key in reqs:
            self.revoking.add(key)

    def apply_answers(self, answers: List[Tuple[tuple, bool]]) -> int:
        """Revoke answers of this step: revoked batches go back to the queue
        FRONT (newest dispatch first, so queue order is kept)."""
        back = []
        for key, revoked in answers:
            self.revoking.discard(key)
            if revoked and key in self.inflight:
                back.append(self.inflight[key])
        for inf in sorted(back, key=lambda i: -i.seq):
            self.inflight.pop(inf.batch.key, None)
            self.jobs.requeue_front(inf.batch.key)
        self.preempted += len(back)
        return len(back)

    # -------------------------------------------------------- complete ----
    def complete(self, key: tuple, service: float = 0.0) -> Optional[Batch]:
        """Batch ``key`` finished and its output is durable. Returns it, or None
        for an unknown / duplicate key."""
        inf = self.inflight.pop(key, None)
        now = time.monotonic()
        self.revoking.discard(key)
        if inf is None or self.jobs.complete(key, now=now) is None:
            return None
        b = inf.batch
        n = len(b.images)
        self.history.append({"job_id": b.job_id, "batch_id": b.batch_id, "model": b.model, "rank": inf.rank,
                             "output": output_name(b.job_id, b.batch_id, self.host_tag)})
        self.metrics.record(b.model, now - inf.t_dispatch, service or now - inf.t_dispatch, n)
        self.cost.observe(b.model, n, service or now - inf.t_dispatch)
        return b

    def requeue_inflight(self) -> int:
        """Failure / growth: every dispatched batch goes back to the FRONT of its
        queue (newest dispatch first, so queue order is preserved)."""
        n = 0
        for inf in sorted(self.inflight.values(), key=lambda i: -i.seq):
            if self.jobs.requeue_front(inf.batch.key) is not None:
                n += 1
        self.inflight.clear()
        self.revoking.clear()
        self.requeued += n
        return n

    def assignments(self) -> Dict[str, dict]:
        """C5: {rank: {model, job_id, batch_id}} — the oldest batch of each rank's queue."""
        out = {}
        for inf in self.inflight.values():
            out.setdefault(f"rank{inf.rank}", {"model": inf.batch.model, "job_id": inf.batch.job_id,
                                               "batch_id": inf.batch.batch_id})
        return out

    def recent(self, n: int = 16, job_id: Optional[int] = None) -> List[dict]:
        """C5 history: the last ``n`` completed batches (of one job) with the rank that ran each."""
        h = [e for e in self.history if job_id is None or e["job_id"] == job_id]
        return h[-n:] if n > 0 else []


# DML_ONE_RANK_SLICE=0: a lone rank runs one model at a time, as the reference's split (A/B)
ONE_RANK_SLICE = os.environ.get("DML_ONE_RANK_SLICE", "1") != "0"
STAGE_DEPTH = int(os.environ.get("DML_STAGE_DEPTH", "8"))  # batches per rank whose images are staged ahead of dispatch (image windows)


def rank_switch_interval() -> None:
    """A rank process runs three Python threads that hand work to each other every batch —
    the serve loop, the control plane's event loop (SWIM, the store, the output PUTs) and the
    output writer. CPython hands the GIL to a waiting thread only every switch interval
    (5 ms by default), so each of those hand-offs could cost milliseconds per batch: 0.5 ms
    (DML_SWITCH_INTERVAL) measured 111 -> 196 batches/s per rank at world 2
    (tools/store_capacity.py, 8-core container)."""
    import sys

    sys.setswitchinterval(float(os.environ.get("DML_SWITCH_INTERVAL", "0.0005")))


def auto_depth(world: int) -> int:
    """Batches in flight per rank (launched, queued, or awaiting their output PUT): 4 on one
    GPU (measured r4, 1 x MI355X, outputs PUT, depth 4 / 8 -> 71.6k / 71.1k images/s at p50
    10.9 / 21.9 ms for ResNet50), 16 with peers: a PUT then replicates to R ranks and the
    step is lockstep over the group, so more batches wait on their output (r5,
    tools/store_capacity.py at world 8 on 8 shared cores: depth 8 / 32 -> 259 / 503 batches/s).
    The image staging look-ahead is STAGE_DEPTH batches per rank whatever the depth (a window
    takes ~10 ms from fetch to resident; at world 1 the depth of 4 left the first pass over new
    images waiting on its windows)."""
    return 4 if world <= 1 else 16


# ---------------------------------------------------------- output writer ----
class OutputWriter:
    """This rank's result files, off the serve loop: a thread renders each
    finished batch (native renderer, byte-identical to the reference's
    indent-4 JSON), writes output_<job>_<batch>_<host>.json into ``out_dir``
    and/or stores it, then calls ``on_written(batch, tag)`` — the service
    reports a batch only after that (reference: PUT, then ACK,
    worker.py:518-537). Storing is pipelined: with ``put_many_async`` the
    finished outputs that are ready are PUT as ONE bundle (up to ``bundle``
    files; store.service.put_many: one leader round trip for all of them) and
    up to ``max_inflight`` bundles are in flight while the next ones render;
    each batch is reported once ITS file is durable (the reference PUT
    fire-and-forget and ACKed at once). ``put`` (one synchronous PUT per file)
    stays for callers without the async path. A write that fails is logged and
    still reported (the job must finish); the failure count is kept."""

    def __init__(self, out_dir: Optional[str], put: Optional[Callable[[str, bytes], None]] = None,
                 host_tag: str = "node", threads: int = 1,
                 put_many_async: Optional[Callable[[List[Tuple[str, bytes]], Callable], None]] = None,
                 bundle: Optional[int] = None, max_inflight: Optional[int] = None):
        self.out_dir, self.put, self.host_tag = out_dir, put, host_tag
        # DML_OUT_BUNDLE / DML_OUT_INFLIGHT: bundle size cap and bundles in flight (A/B)
        bundle = bundle or int(os.environ.get("DML_OUT_BUNDLE", "16"))
        max_inflight = max_inflight or int(os.environ.get("DML_OUT_INFLIGHT", "4"))
        self.put_many_async, self.bundle = put_many_async, max(1, bundle)
        if out_dir:
            os.makedirs(out_dir, exist_ok=True)
        self.renderer = BatchRenderer()   # thread-safe: per-thread scratch buffers
        self.q: "queue.Queue" = queue.Queue()
        self.written = 0
        self.failed = 0
        self.bytes = 0
        self.busy_s = 0.0
        self.bundles = 0
        self._slots = threading.BoundedSemaphore(max(1, max_inflight))
        self._cv = threading.Condition()
        self._inflight = 0
        self._threads = [threading.Thread(target=self._loop, daemon=True, name=f"output-writer-{i}")
                         for i in range(threads)]
        for t in self._threads:
            t.start()

    @property
    def enabled(self) -> bool:
        return bool(self.out_dir) or self.put is not None or self.put_many_async is not None

    def submit(self, b: Batch, idx: np.ndarray, p: np.ndarray, grank: int,
               on_written: Optional[Callable[..., None]] = None, tag=None) -> None:
        self.q.put((b, idx, p, grank, on_written, tag))

    def _render(self, item) -> Optional[Tuple[str, bytes]]:
        b, idx, p, g, _, _ = item
        try:
            data = self.renderer.render(b.images, idx, p)
            # one name per (job, batch) whichever rank ran it: a batch re-run after a rank
            # died between storing its output and reporting it writes a new VERSION of the
            # same file, so every output exists exactly once in the store
            name = output_name(b.job_id, b.batch_id, self.host_tag)
            if self.out_dir:
                with open(os.path.join(self.out_dir, name), "wb") as f:
                    f.write(data)
            self.bytes += len(data)
            return name, data
        except Exception as e:  # a failed write is logged, never silently skipped
            self.failed += 1
            log.error("output %s:%s not written: %s", b.job_id, b.batch_id, e)
            return None

    @staticmethod
    def _report(item) -> None:
        b, _, _, _, on_written, tag = item
        if on_written is not None:
            on_written(b, tag)

    def _loop(self) -> None:
        while True:
            first = self.q.get()
            if first is None:
                self.q.task_done()
                return
            items, stop = [first], False
            if self.put_many_async is not None:  # every ready output joins the bundle
                while len(items) < self.bundle:
                    try:
                        it = self.q.get_nowait()
                    except queue.Empty:
                        break
                    if it is None:
                        stop = True
                        break
                    items.append(it)
            t0 = time.perf_counter()
            rendered = [self._render(it) for it in items]
            if self.put_many_async is not None:
                ok_items = [(it, r) for it, r in zip(items, rendered) if r is not None]
                for it, r in zip(items, rendered):
                    if r is None:
                        self._report(it)
                if ok_items:
                    self._slots.acquire()   # at most max_inflight bundles in flight
                    with self._cv:
                        self._inflight += 1
                    self.bundles += 1
                    self.put_many_async([r for _, r in ok_items],
                                        lambda ok, bad, ok_items=ok_items: self._bundle_done(ok_items, bad))
            else:
                for it, r in zip(items, rendered):
                    if r is not None:
                        try:
                            if self.put is not None:
                                self.put(*r)
                            self.written += 1
                        except Exception as e:
                            self.failed += 1
                            log.error("output %s not stored: %s", r[0], e)
                    self._report(it)
            self.busy_s += time.perf_counter() - t0
            for _ in items:
                self.q.task_done()
            if stop:
                self.q.task_done()
                return

    def _bundle_done(self, ok_items, failed_names) -> None:
        """(the store's thread) a bundle's PUT finished: report its batches."""
        bad = set(failed_names)
        for it, (name, _) in ok_items:
            if name in bad:
                self.failed += 1
                log.error("output %s not stored", name)
            else:
                self.written += 1
            self._report(it)
        with self._cv:
            self._inflight -= 1
            self._cv.notify_all()
        self._slots.release()

    def flush(self, timeout: float = 300.0) -> None:
        """Block until every queued file is written and every bundle is durable."""
        self.q.join()
        with self._cv:
            self._cv.wait_for(lambda: self._inflight == 0, timeout)

    def close(self) -> None:
        for _ in self._threads:
            self.q.put(None)
        for t in self._threads:
            t.join(timeout=10)


# ---------------------------------------------------------------- service ----
@dataclass
class _Launched:
    batch: Batch
    rows: object            # [2, cap, 5] int32: a torch tensor or a numpy view (no torch call per poll)
    event: Optional[object]
    slot: int
    t0: float
    epoch: int


class CollectiveService:
    """The per-rank serve loop (identical on every rank). See the module doc.

    ``control``: optional RankControl (UDP control plane + store of this rank);
    without it (tests, benches) jobs are submitted with ``submit_local`` on the
    coordinator rank. ``writer``: this rank's OutputWriter (None: batches are
    reported as soon as their GPU work finishes, no files). ``rejoined``: this
    process re-joined a running job (its replica is empty until the
    coordinator's state record)."""

    def __init__(self, eg: ElasticGroup, backend: RankBackend, coord: ReplicatedCoordinator,
                 control=None, writer: Optional[OutputWriter] = None, kill_rank: int = -1, kill_at_step: int = -1,
                 on_device: bool = False, idle_sleep: float = 0.002, poll_sleep: float = 0.0002,
                 watchdog_s: float = 0.0, rejoined: bool = False, kill_at_done: int = -1,
                 stall: Tuple[int, int, float] = (-1, -1, 0.0)):
        self.eg, self.be, self.coord, self.control = eg, backend, coord, control
        # fault injection (tests): (rank, step, seconds) - that rank's serve loop AND control
        # plane freeze for that long at that step, alive but silent (a false SWIM suspicion)
        self.stall = stall
        self.writer = writer
        # fault injection (tests, BASELINE config 5): rank kill_rank exits 17 at step
        # kill_at_step, or once kill_at_done batches have completed (replicated count)
        self.kill_rank, self.kill_at_step, self.kill_at_done = kill_rank, kill_at_step, kill_at_done
        self.completed = 0
        # recovery timing: from the last step completed before a failure (a killed rank dies
        # right after its last step) to the first step after the rebuild that dispatched work
        self.last_ok_t = time.monotonic()
        self._recovering_since: Optional[float] = None
        self.recoveries_s: List[float] = []
        self.dev = backend.device if on_device else torch.device("cpu")
        self.steps = 0
        self.rebuilds = 0
        self.grows = 0
        self.rejoins = 0   # times this live rank was removed and re-admitted (false suspicion)
        self._frozen = False
        self.cap = backend.cap
        self.slots = getattr(backend, "slots", SLOTS)
        self.hostq: "deque[Batch]" = deque()             # dispatched to this rank, not launched
        self.gpu: "deque[_Launched]" = deque()           # launched, not finished (launch order)
        self.free_slots = list(range(self.slots))
        # finished + written: (batch, service s, epoch, top-5 ids [n, 5] int32, probs [n, 5] fp32)
        self.done: "deque[tuple]" = deque()
        # the result collect (SURVEY §2.6 "gather: results"): each rank's reported batches' packed
        # top-5 rows (40 B per image) go to the coordinator by a gather on the epoch's result group
        # (RCCL over xGMI on a GPU node). Ranks hold their rows until some rank has
        # ``collect_every`` reports pending, a job has finished, or the service stops: the
        # coordinator decides and sets F_FLUSH in its record, so every rank flushes on the same
        # step, with the same buffer shape (read off the step's exchange). The
        # coordinator keeps the rows per job, so get-output renders final_<job>.json once from
        # them (RankControl GET_OUTPUT) instead of listing and fetching every output file from
        # the store. DML_COLLECT_RESULTS=0: off (the same value on every rank).
        self.collect = os.environ.get("DML_COLLECT_RESULTS", "1") != "0"
        # ~8k images a flush (32 b256 batches; 40 B an image, 320 KiB a rank's buffer)
        self.collect_every = max(1, int(os.environ.get("DML_COLLECT_EVERY", "0")) or 8192 // max(1, backend.cap))
        self.collect_flushes = 0
        # DML_COLLECT_FORCE_GATHER=1: gather over the result group at world 1 too (a one-rank
        # RCCL gather: the GPU test of the collective path on a one-GPU box)
        self._force_gather = os.environ.get("DML_COLLECT_FORCE_GATHER") == "1"
        self._pend_epoch = -1
        self._pend_rows: List[tuple] = []              # this rank's reports since the last flush
        self._pend_keys: List[List[tuple]] = []        # per group rank: the (job, batch) keys it reported
        self._pend_imgs: Dict[tuple, list] = {}        # (coordinator) finished batch -> its image names
        # gathers in flight, oldest first: (work, done-event or None, tensors kept alive, host rows
        # on the coordinator, keys, images); drained each step, so a flush never blocks the loop
        self._gathers: "deque[tuple]" = deque()
        self._flush_due = False
        self.results: "OrderedDict[int, Dict[int, tuple]]" = OrderedDict()   # job -> batch -> (images, ids, probs)
        self.results_jobs_max = 64
        self.collected_rows = 0
        self._results_lock = threading.Lock()   # the serve loop inserts, the control loop renders
        self.answers: List[Tuple[tuple, bool]] = []       # revoke answers for the next record
        self.launched = 0
        self.served_here = 0
        self.idle_sleep, self.poll_sleep = idle_sleep, poll_sleep
        self._inbox: "queue.Queue" = queue.Queue()   # (record, reply callback or None)
        self._stop = False
        self.rejoined = rejoined
        # ranks whose replica has not yet received a coordinator state record (a re-joined
        # process, until the first state record of its epoch): never the coordinator
        self.unsynced: set = {eg.grank} if rejoined else set()
        if rejoined:
            self.unsynced |= set(eg.members) - set(eg.prev_members)
        # queued batches staged ahead of dispatch (the in-flight ones are staged besides)
        self.stage_ahead = max(1, eg.world) * STAGE_DEPTH
        self._rec_bufs: Dict[tuple, object] = {}   # the step's exchange output, per (world, L)
        # a staging backend (image arenas): queued batches get an affinity rank, their images
        # are staged there ahead of dispatch and the plan sends them there
        self._targeted = hasattr(backend, "arenas")
        self.last_progress = time.monotonic()
        self.phase_s: Dict[str, float] = {"poll": 0.0, "plan": 0.0, "collective": 0.0, "apply": 0.0,
                                          "launch": 0.0, "sleep": 0.0}
        self.phase_max: Dict[str, float] = dict.fromkeys(self.phase_s, 0.0)   # the longest single step part
        self.batches_per_step_max = 0
        self._watchdog = None
        if watchdog_s > 0:
            self._watchdog = threading.Thread(target=self._watch, args=(watchdog_s,), daemon=True)
            self._watchdog.start()
        if control is not None:
            control.attach(self)
        backend.attach(eg)
        # RCCL creates a communicator at its first collective (seconds on a cold node): a first
        # flush at a job's end then held the serve loop, and get-output fell back to the files.
        # Every rank builds its service at the same point, so the result group's communicator is
        # made here (a re-joining rank skips it: the survivors are serving; its new epoch's group
        # comes up at that epoch's first flush, on every member at once)
        if (self.collect and not rejoined and getattr(eg, "data_backend", "gloo") == "nccl"
                and getattr(eg, "result_group", None) is not None and (eg.world > 1 or self._force_gather)
                and self.be.device.type == "cuda"):
            t = torch.zeros((1, 1, 10), dtype=torch.int32, device=self.be.device)
            eg.gather_result(t, [torch.empty_like(t) for _ in range(eg.world)] if eg.rank == 0 else None, 0)
            torch.cuda.synchronize(self.be.device)

    # ------------------------------------------------------------- roles --
    def coordinator_rank(self) -> int:
        """The highest member whose replica is in sync (a re-joined rank with a higher id
        would otherwise plan from an empty replica: ADVICE r3)."""
        synced = [g for g in self.eg.members if g not in self.unsynced]
        return max(synced or self.eg.members)

    def is_coordinator(self) -> bool:
        return self.eg.grank == self.coordinator_rank()

    # ------------------------------------------------------------ inputs --
    def submit_local(self, model: str, n_images: int = 0, images: Optional[List[str]] = None,
                     requester: str = "local", reply: Optional[Callable[[dict], None]] = None) -> None:
        """Queue a submit on the coordinator (applied at the next step)."""
        names = list(images) if images is not None else synthetic_names(n_images)   # lazy: two ints
        self._inbox.put(({"op": "submit", "model": model, "images": names, "requester": requester}, reply))

    def set_batch_size(self, model: str, bs: int, reply: Optional[Callable[[dict], None]] = None) -> None:
        self._inbox.put(({"op": "batch_size", "model": model, "batch_size": int(bs)}, reply))

    def stop(self) -> None:
        self._stop = True

    def _drain(self) -> Tuple[List[dict], List[Optional[Callable]]]:
        recs, replies = [], []
        while True:
            try:
                rec, reply = self._inbox.get_nowait()
            except queue.Empty:
                break
            if rec["op"] == "submit":
                rec["job_id"] = self.coord.next_job_id(sum(r["op"] == "submit" for r in recs))
            recs.append(rec)
            replies.append(reply)
        return recs, replies

    # ----------------------------------------------------------- own work --
    def _written(self, b: Batch, tag) -> None:
        """(writer thread) output durable: reportable at the next step."""
        self.done.append((b, tag[0], tag[1], tag[2], tag[3]))

    def _poll(self) -> int:
        """Finished GPU batches -> writer (or straight to the report list);
        launch host-queued batches into free slots. Never blocks."""
        n = 0
        while self.gpu:
            L = self.gpu[0]
            if L.event is not None and not L.event.query():
                break
            self.gpu.popleft()
            self.be.finalize(L.slot)
            svc = time.monotonic() - L.t0
            k = len(L.batch.images)
            rows = L.rows[:, :k] if isinstance(L.rows, np.ndarray) else L.rows[:, :k].numpy()
            idx = rows[0].copy()
            p = rows[1].view(np.float32).copy()
            self.free_slots.append(L.slot)
            if self.writer is not None and self.writer.enabled:
                self.writer.submit(L.batch, idx, p, self.eg.grank, on_written=self._written,
                                   tag=(svc, L.epoch, idx, p))
            else:
                self.done.append((L.batch, svc, L.epoch, idx, p))
            self.served_here += 1
            n += 1
        self.be.progress()  # image windows: decode shares, all-gathers, scatters (never blocks)
        while self.hostq and self.free_slots and self.be.ready(self.hostq[0].model, self.hostq[0].images):
            b = self.hostq.popleft()
            slot = self.free_slots.pop(0)
            rows, ev = self.be.launch(b.model, b.images, slot)
            self.gpu.append(_Launched(b, rows, ev, slot, time.monotonic(), self.eg.epoch))
            self.launched += 1
            n += 1
        return n

    # -------------------------------------------------------------- step --
    def _record(self, L: int, depth: int, active: bool, loglen: int, stop: bool, grow: List[int],
                table: Optional[np.ndarray], reqs: List[Tuple[int, tuple]]) -> Tuple[np.ndarray, list, list]:
        world = self.eg.world
        tab, req, rep, ack = _offs(world, depth)
        r = np.zeros(L, np.int64)
        r[H_VALID] = 1
        reports = []
        while self.done and len(reports) < RP_MAX:
            b, svc, ep, ids, probs = self.done.popleft()
            if ep != self.eg.epoch:
                continue  # requeued by a rebuild since: it runs again
            reports.append((b, svc, ids, probs))
        answers, self.answers = self.answers[:RV_MAX], self.answers[RV_MAX:]
        r[H_NREP] = len(reports)
        for i, (b, svc, _, _) in enumerate(reports):
            r[rep + i * REP_W: rep + (i + 1) * REP_W] = (b.job_id, b.batch_id, int(svc * 1e6), b.attempts)
        r[H_NACK] = len(answers)
        for i, (key, ok) in enumerate(answers):
            r[ack + i * ACK_W: ack + (i + 1) * ACK_W] = (key[0], key[1], int(ok))
        if active:
            r[H_LOGLEN] = loglen
            r[H_STEP] = self.steps
            r[H_FLAGS] = (F_STOP if stop else 0) | (F_GROW if grow else 0) | (F_FLUSH if self._flush_wanted(stop) else 0)
            r[H_GROW] = sum(1 << g for g in grow)
            if table is not None:
                r[tab:req] = table.reshape(-1)
            else:
                r[tab:req] = -1
            r[H_NREQ] = len(reqs)
            for i, (g, key) in enumerate(reqs):
                r[req + i * REQ_W: req + (i + 1) * REQ_W] = (g, key[0], key[1])
        return r, reports, answers

    def step(self, stop_when_idle: bool = False) -> bool:
        eg, coord = self.eg, self.coord
        world, depth = eg.world, coord.depth
        L = rec_len(world, depth)
        tab, req, rep, ack = _offs(world, depth)
        root = eg.group_rank_of(self.coordinator_rank())
        ph, pm, t0 = self.phase_s, self.phase_max, time.perf_counter()
        moved0 = self._poll()
        t1 = time.perf_counter()
        ph["poll"] += t1 - t0
        pm["poll"] = max(pm["poll"], t1 - t0)
        active = self.is_coordinator()
        payload, recs, replies, results = b"", [], [], []
        table, reqs, grow, stop = None, [], [], False
        if active:
            recs, replies = self._drain()
            with coord.lock:
                results = [coord.apply(r) for r in recs]  # the coordinator applies its log first, like everyone
                stop = self._stop or (stop_when_idle and coord.idle() and not recs)
                if not stop:
                    grow = sorted(g for g in set(eg.joiners) if g not in eg.members)
                    if grow:
                        grow = [g for g in eg.admit(set(grow)) if g not in eg.members]
                    if not grow:
                        disp, reqs = coord.plan(eg.members)
                        table = coord.table(eg.members, disp)
            if recs:
                payload = json.dumps(recs, default=json_default).encode()
        rec, reports, answers = self._record(L, depth, active, len(payload), stop, grow, table, reqs)
        t2 = time.perf_counter()
        ph["plan"] += t2 - t1
        pm["plan"] = max(pm["plan"], t2 - t1)
        # ---- the step's collective (+ the log bytes, rarely) ----
        # host path (shared-memory exchange): numpy end to end — every torch call on the serve
        # loop hands the GIL to the rank's writer / control threads and waits to get it back
        # (measured: 0.2-0.5 ms per trivial tensor op at world 8)
        host = self.dev.type == "cpu"
        out = self._rec_bufs.get((world, L))
        if out is None:  # one buffer per group shape: no allocation per step
            out = self._rec_bufs[(world, L)] = (np.empty((world, L), np.int64) if host else
                                                torch.empty((world, L), dtype=torch.int64, device=self.dev))
        applied_here: List[dict] = []
        try:
            if world == 1:  # nothing to exchange: a collective would only hand the GIL around
                h = rec[None]
                n = 0
            else:
                if host:
                    eg.exchange(out, rec, root)
                    h = out
                else:
                    eg.exchange(out, torch.from_numpy(rec).to(self.dev), root)
                    h = out.cpu().numpy()
                n = int(h[root, H_LOGLEN])
            if n:
                got = eg.broadcast_bytes(payload if active else None, n, src=root)
                if not active:
                    applied_here = json.loads(got.decode())
        except CollectiveFailure:
            # nothing of this step was applied anywhere: its reports and answers go again
            for b, svc, ids, probs in reversed(reports):
                self.done.appendleft((b, svc, self.eg.epoch, ids, probs))
            self.answers = answers + self.answers
            raise
        t3 = time.perf_counter()
        ph["collective"] += t3 - t2
        pm["collective"] = max(pm["collective"], t3 - t2)
        # ---- apply, in the same order on every rank: log, reports, answers, table ----
        with coord.lock:
            for r in applied_here:
                coord.apply(r)
        applied = recs if active else applied_here
        for r in applied:
            if r["op"] == "state":  # every replica now holds the coordinator's state
                self.rejoined = False
                self.unsynced.clear()
        if active and self.control is not None:
            self.control.committed(replies, results)
        elif active:
            for cb, r in zip(replies, results):
                if cb is not None:
                    cb(r)
        flags = int(h[root, H_FLAGS])
        finished: List[Batch] = []
        moved = 0
        rq: List[Tuple[int, tuple]] = []
        mine: Optional[List[Batch]] = None
        with coord.lock:
            for r in range(world):
                for i in range(int(h[r, H_NREP])):
                    j, bt, us, _ = h[r, rep + i * REP_W: rep + (i + 1) * REP_W]
                    b = coord.complete((int(j), int(bt)), service=int(us) * 1e-6)
                    if b is not None:
                        finished.append(b)
                        self.be.release(b.model, b.key, b.images)  # its images are no longer pinned
            ans = []
            for r in range(world):
                for i in range(int(h[r, H_NACK])):
                    j, bt, ok = h[r, ack + i * ACK_W: ack + (i + 1) * ACK_W]
                    ans.append(((int(j), int(bt)), bool(ok)))
            coord.apply_answers(ans)
            if not flags & F_STOP:
                table = h[root, tab:req].reshape(world, depth, TAB_W)
                disp = coord.apply_table(table, eg.members)
                mine = disp.get(eg.grank, [])
                moved = sum(len(v) for v in disp.values())
                rq = [(int(h[root, req + i * REQ_W]), (int(h[root, req + i * REQ_W + 1]),
                                                       int(h[root, req + i * REQ_W + 2])))
                      for i in range(int(h[root, H_NREQ]))]
                coord.apply_requests(rq)
                self._stage()
        if self.collect:
            try:
                self._collect(h, rep, world, root, active, reports, finished, bool(flags & F_FLUSH))
            except CollectiveFailure:
                raise
            except Exception as e:   # the same code on every rank: it fails everywhere alike
                log.error("rank %d: result collect disabled: %s", eg.grank, e)
                self.collect = False
                self._gathers.clear()
        if finished and active and self.control is not None:
            self.control.jobs_progress(finished)
        t4 = time.perf_counter()
        ph["apply"] += t4 - t3
        pm["apply"] = max(pm["apply"], t4 - t3)
        if mine is None:  # STOP (sent only when nothing is queued or in flight)
            return False
        self.batches_per_step_max = max(self.batches_per_step_max, moved)
        now = time.monotonic()
        if self._recovering_since is not None and moved:
            self.recoveries_s.append(now - self._recovering_since)
            self._recovering_since = None
        self.last_ok_t = now
        self.completed += len(finished)
        if eg.grank == self.kill_rank and (self.steps == self.kill_at_step or
                                           0 <= self.kill_at_done <= self.completed):
            log.warning("rank %d: injected kill at step %d (%d batches done)", eg.grank, self.steps, self.completed)
            os._exit(17)
        if eg.grank == self.stall[0] and self.steps == self.stall[1]:
            log.warning("rank %d: injected stall of %.1f s at step %d", eg.grank, self.stall[2], self.steps)
            if self.control is not None and self.control.loop is not None:
                self.control.loop.call_soon_threadsafe(time.sleep, self.stall[2])
            time.sleep(self.stall[2])
        # own new batches, then the revoke requests addressed to this rank (host queue only)
        self.hostq.extend(mine)
        for g, key in rq:
            if g != eg.grank:
                continue
            hit = next((b for b in self.hostq if b.key == key), None)
            if hit is not None:
                self.hostq.remove(hit)
            self.answers.append((key, hit is not None))
        if flags & F_GROW:
            self._grow([g for g in range(63) if (int(h[root, H_GROW]) >> g) & 1])
        moved0 += self._poll()
        self.steps += 1
        if os.environ.get("DML_SVC_DEBUG") and self.steps % 200 == 0:
            log.warning("rank %d step %d epoch %d: queued %s inflight %d hostq %d gpu %d done %d root %d",
                        eg.grank, self.steps, eg.epoch, {m: len(q) for m, q in coord.jobs.queues.items()},
                        len(coord.inflight), len(self.hostq), len(self.gpu), len(self.done), root)
        self.last_progress = time.monotonic()
        t5 = time.perf_counter()
        ph["launch"] += t5 - t4
        pm["launch"] = max(pm["launch"], t5 - t4)
        if not (reports or answers or mine or n or self.done or self.answers or self.gpu or self.hostq):
            time.sleep(self.poll_sleep if coord.inflight else self.idle_sleep)
            ph["sleep"] += time.perf_counter() - t5
        elif world == 1 and not (moved0 or reports or answers or mine or n):
            # world 1 has no exchange to block in: a step that moved nothing (batches waiting on
            # the GPU or on their image window) would otherwise spin in Python and hold the GIL
            # against the decode pool, the writer and the control loop (measured: a store-image
            # window's fetch took 60-110 s behind such a spin, 32 decode threads)
            time.sleep(self.poll_sleep)
            ph["sleep"] += time.perf_counter() - t5
        return True

    def _collect(self, h: np.ndarray, rep: int, world: int, root: int, active: bool, reports: list,
                 finished: List[Batch], flush: bool) -> None:
        """Queue the step's reported rows; on a flush step gather every rank's queued rows to
        the coordinator (same step, same [k, cap, 10] int32 shape everywhere: k and the flush
        decision come from the step's exchange, which every rank holds identically)."""
        if self._pend_epoch != self.eg.epoch:   # a new group: every member starts empty
            self._pend_epoch = self.eg.epoch
            self._pend_rows, self._pend_imgs = [], {}
            self._pend_keys = [[] for _ in range(world)]
            self._gathers.clear()               # the old group's gathers died with it
        self._drain_gathers()
        nreps = h[:, H_NREP].tolist()
        for r in range(world):
            if nreps[r]:
                v = h[r, rep: rep + nreps[r] * REP_W].tolist()
                self._pend_keys[r].extend(zip(v[0::REP_W], v[1::REP_W]))
        for b, _, ids, probs in reports:
            self._pend_rows.append((len(b.images), ids, probs))
        if active:
            for b in finished:
                self._pend_imgs[b.key] = b.images   # a batch's names are never mutated (lazy for synthetic jobs)
                j = self.coord.jobs.jobs.get(b.key[0])
                if j is not None and j.done:
                    self._flush_due = True   # get-output of that job wants its last rows
        k = max(len(p) for p in self._pend_keys)
        if k == 0 or not flush:
            return
        self._flush_due = False
        buf = np.zeros((k, self.cap, 10), np.int32)
        for i, (n, ids, probs) in enumerate(self._pend_rows):
            if ids is None or not n:
                buf[i, :, 0] = -1        # no rows for this report: the coordinator skips it
                continue
            buf[i, :n, :5] = ids[:n]
            buf[i, :n, 5:] = np.ascontiguousarray(probs[:n], dtype=np.float32).view(np.int32)
        keys, imgs = self._pend_keys, self._pend_imgs
        self._pend_rows, self._pend_imgs = [], {}
        self._pend_keys = [[] for _ in range(world)]
        self.collect_flushes += 1
        if world == 1 and not self._force_gather:
            self._take_rows([buf], keys, imgs)
            return
        if getattr(self.eg, "data_backend", "gloo") == "nccl":
            # a side stream: the gather and the coordinator's device->host copy wait for each
            # other only, not for the model work queued on the serving streams
            # the backend's GPU (the control group may be gloo, with no device of its own: the
            # bench's service passes run --comm gloo with an RCCL data group)
            dev = self.be.device
            st = getattr(self, "_collect_stream", None)
            if st is None:
                st = self._collect_stream = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(st):
                t = torch.from_numpy(buf).to(dev)
                outs = [torch.empty_like(t) for _ in range(world)] if self.eg.rank == root else None
                w = self.eg.gather_result_async(t, outs, root)
                host, ev = None, None
                if active:
                    w.wait()   # stream-ordered: the copies below run after the gather
                    host = torch.empty((world,) + tuple(buf.shape), dtype=torch.int32, pin_memory=True)
                    for r in range(world):
                        host[r].copy_(outs[r], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(st)
            self._gathers.append((w, ev, (t, outs), host, keys if active else None, imgs))
        else:
            t = torch.from_numpy(buf)
            outs = [torch.empty_like(t) for _ in range(world)] if self.eg.rank == root else None
            w = self.eg.gather_result_async(t, outs, root)
            self._gathers.append((w, None, (t, outs), outs if active else None, keys if active else None, imgs))

    def _flush_wanted(self, stop: bool) -> bool:
        """(coordinator, building its record) flush the result rows this step?"""
        if not self.collect or not self._pend_keys:
            return False
        return stop or self._flush_due or max(len(p) for p in self._pend_keys) >= self.collect_every

    def _drain_gathers(self, block: bool = False, limit_s: float = 30.0) -> None:
        """Apply the finished result gathers, oldest first (``block``: wait for all of them, at
        most ``limit_s``: the end of ``serve``; a gather still pending then is dropped, and
        get-output for its batches falls back to the output files)."""
        end = time.monotonic() + limit_s
        while self._gathers:
            w, ev, _, host, keys, imgs = self._gathers[0]
            if not (ev.query() if ev is not None else w.is_completed()):
                if not block:
                    return
                if time.monotonic() > end:
                    log.warning("rank %d: %d result gathers still pending at the end of serve; dropped",
                                self.eg.grank, len(self._gathers))
                    self._gathers.clear()
                    return
                time.sleep(0.001)
                continue
            self._gathers.popleft()
            try:
                if ev is not None:
                    ev.synchronize()
                else:
                    w.wait()
            except Exception as e:   # the group failed under it: those batches fall back to the files
                log.warning("result gather failed: %s", e)
                continue
            if keys is not None:
                # (pinned staging is copied out once: the kept rows must not pin host memory)
                got = host.numpy().copy() if ev is not None else [o.numpy() for o in host]
                self._take_rows(got, keys, imgs)

    def _take_rows(self, got, keys: List[List[tuple]], imgs: Dict[tuple, list]) -> None:
        for r in range(len(keys)):
            for i, key in enumerate(keys[r]):
                names = imgs.pop(key, None)
                if names is None:   # a duplicate report (a re-run batch): the first one counted
                    continue
                rows = got[r][i, :len(names)]
                if rows.shape[0] == 0 or rows[0, 0] < 0:
                    continue
                with self._results_lock:
                    per = self.results.get(key[0])
                    if per is None:
                        per = self.results[key[0]] = {}
                        while len(self.results) > self.results_jobs_max:
                            self.results.popitem(last=False)
                    per[key[1]] = (names, rows[:, :5], rows[:, 5:].view(np.float32))   # views of the gathered buffer
                self.collected_rows += len(names)

    def final_output(self, job_id: int, host_tag: str, wait_s: float = 0.0) -> Optional[bytes]:
        """(coordinator) final_<job>.json from the gathered rows, byte-identical to get-output's
        merge of the job's output files in store-listing order (worker.py:1617-1627); None until
        every batch of the job has been collected here."""
        from ..serving.output import output_name
        end = time.monotonic() + wait_s   # a just-finished job's last rows flush within a few steps
        while True:
            with self.coord.lock:
                j = self.coord.jobs.jobs.get(job_id)
                total = j.batches_total if j is not None else -1
            with self._results_lock:
                per = dict(self.results.get(job_id) or {})
            if per and total >= 0 and len(per) == total:
                break
            if time.monotonic() >= end or j is None or not j.done:
                return None
            time.sleep(0.01)
        order = sorted(per, key=lambda bt: output_name(job_id, bt, host_tag))
        return self._renderer().render_merged([per[bt] for bt in order])

    def _renderer(self):
        r = getattr(self, "_render", None)
        if r is None:
            from ..serving.output import BatchRenderer
            r = self._render = BatchRenderer()
        return r

    def _stage(self) -> None:
        """(every rank, same step, coordinator lock held) stage the images of the batches
        in flight - for the rank running each - and of the next ``stage_ahead`` queued
        batches of each model - for their affinity rank - in dispatch order
        (parallel/image_store.py): identical decisions everywhere."""
        coord = self.coord
        members = self.eg.members
        for m in MODELS:
            cand, where = [], {}
            for inf in coord.inflight.values():
                if inf.batch.model == m:
                    cand.append(inf.batch)
                    where[inf.batch.key] = inf.rank
            if self._targeted:
                ahead = list(islice(coord.jobs.queues[m], 0, self.stage_ahead))
                aff = coord.assign_affinity(m, ahead, members)
                for b in ahead:
                    g = aff.get(b.key)
                    if g is not None:
                        cand.append(b)
                        where[b.key] = g
            if cand:
                self.be.stage(m, cand, where)

    # -------------------------------------------------------------- serve --
    def freeze_heap(self) -> None:
        """Everything set up so far (torch, the engines, the arenas' bookkeeping) is
        long-lived: moved out of the cyclic collector's generations, a full collection no
        longer walks it (measured ~100 ms per pass over ~175k objects with the GIL held -
        every thread of the rank, its SWIM acks included, stalls for it). Once per process;
        serve() calls it if the caller did not (benches call it before their timer)."""
        if not self._frozen:
            gc.collect()
            gc.freeze()
            # young-generation passes 100x rarer than CPython's default (700, 10, 10): the serve
            # loop's garbage is acyclic (freed by refcount), and every pass holds the GIL on a
            # lockstep rank (world-8 capacity 2500 -> 2614 batches/s, profiles/r5_rr);
            # DML_GC_THRESHOLD=<g0,g1,g2> overrides (A/B)
            th = os.environ.get("DML_GC_THRESHOLD", "100000,50,1000")
            gc.set_threshold(*(int(v) for v in th.split(",")))
            self._frozen = True

    def serve(self, max_steps: int = 10 ** 9, stop_when_idle: bool = False, deadline: Optional[float] = None) -> int:
        """Run steps until STOP (stop_when_idle: once every job is done) or ``max_steps``.
        ``deadline`` (time.monotonic()): raise TimeoutError past it (a bench pass with a time
        budget; the product runs without one)."""
        self.freeze_heap()
        while self.steps < max_steps:
            if deadline is not None and time.monotonic() > deadline:
                raise TimeoutError(f"rank {self.eg.grank}: serve deadline passed at step {self.steps}")
            try:
                if not self.step(stop_when_idle):
                    break
            except CollectiveFailure as e:
                self._recover(e)
        self._drain_gathers(block=True)
        self.be.drain()
        if self.writer is not None:
            self.writer.flush()
        return self.steps

    def _reset_local(self) -> None:
        """Drop this rank's queue and in-flight work (requeued everywhere)."""
        with self.coord.lock:
            self.coord.requeue_inflight()
        self.be.drain()   # the requeued batches' GPU work may still run: let it finish before slots are reused
        self.hostq.clear()
        self.gpu.clear()
        self.free_slots = list(range(self.slots))
        self.answers = []

    def _after_epoch(self, was: int) -> None:
        # ranks new in this epoch (re-joined) and ranks still waiting for their first state
        # stay out of the coordinator role until the next state record
        self.unsynced = (self.unsynced & set(self.eg.members)) | (set(self.eg.members) - set(self.eg.prev_members))
        self.stage_ahead = self.eg.world * STAGE_DEPTH
        # image windows: every rank forgets its staging at this same boundary and stages
        # afresh over the new group (a joiner's arena is empty; survivors' collectives of
        # the failed epoch were aborted)
        self.be.reset_staging()
        with self.coord.lock:
            self.coord.reset_affinity()
        self.be.attach(self.eg)
        # the new coordinator's state is authoritative: replicas that completed one
        # step more or less than it did are repaired by a state record (and a
        # joiner gets its first state); it is the first record of the next step
        if self.is_coordinator():
            with self.coord.lock:
                snap = self.coord.jobs.snapshot()
            with self._inbox.mutex:
                self._inbox.queue.appendleft(({"op": "state", "jobs": snap}, None))
            if self.control is not None and was != self.eg.grank:
                self.control.became_coordinator(was)
        self.last_progress = time.monotonic()

    def _recover(self, e: Exception) -> None:
        eg = self.eg
        log.warning("rank %d: collective failed (%s); rebuilding", eg.grank, e)
        if self._recovering_since is None:
            self._recovering_since = self.last_ok_t
        was = self.coordinator_rank()
        self._reset_local()
        if "removed from the group" in str(e) and self.control is not None:
            self._rejoin_alive()  # the others fixed the next epoch without this (live) rank
            return
        for attempt in range(5):
            deadline = time.monotonic() + 10
            while not (eg.dead & set(eg.members)) and time.monotonic() < deadline:
                time.sleep(0.01)  # let SWIM confirm who died
            try:
                eg.rebuild(set(eg.dead))  # aborts the communicator first (RCCL: ncclCommAbort)
                break
            except CollectiveFailure as e2:
                if "removed from the group" in str(e2) and self.control is not None:
                    self._rejoin_alive()
                    return
                if "removed from the group" in str(e2) or attempt == 4:
                    raise
                log.warning("rank %d: rebuild failed (%s); retrying with the updated dead set", eg.grank, e2)
        self.rebuilds += 1
        self._after_epoch(was)

    def _rejoin_alive(self) -> None:
        """The others removed this live rank (SWIM suspected it past the timeout while it was
        stalled). Its control plane refutes the suspicion, the coordinator admits it again
        (a SWIM rejoin), and it re-enters as a re-joined process: replica empty until the
        coordinator's state record, its queued and in-flight work already requeued."""
        eg = self.eg
        log.warning("rank %d: removed from the group while alive; waiting for re-admission", eg.grank)
        was = self.coordinator_rank()
        eg.rejoin(timeout_s=120.0)
        self.rejoined = True
        self.unsynced = {eg.grank} | (set(eg.members) - set(eg.prev_members))
        self.done.clear()   # reports of the epoch this rank left: requeued by the others
        self.rejoins += 1
        self._after_epoch(was)

    def _grow(self, joiners: List[int]) -> None:
        """Admit re-joined ranks (every member, at the same step boundary)."""
        eg = self.eg
        was = self.coordinator_rank()
        log.warning("rank %d: admitting ranks %s into epoch %d", eg.grank, joiners, eg.epoch + 1)
        self._reset_local()
        try:
            eg.grow(sorted(set(eg.members) | set(joiners)))
        except CollectiveFailure:
            raise
        except Exception as e:  # a joiner that never arrived (it died again): rebuild without it
            raise CollectiveFailure(f"epoch {eg.epoch} growth failed: {e}") from e
        self.grows += 1
        self._after_epoch(was)

    def _watch(self, limit_s: float) -> None:
        """Watchdog: a rank whose serve loop makes no progress for ``limit_s``
        (e.g. stuck inside a collective the abort could not release) exits
        non-zero; it is never re-exec'ed (the survivors rebuild without it)."""
        while True:
            time.sleep(min(1.0, limit_s / 4))
            if time.monotonic() - self.last_progress > limit_s:
                log.error("rank %d: no progress for %.0f s, exiting", self.eg.grank, limit_s)
                os._exit(3)


# control plane of a rank (kept importable from here)
from .rank_control import RankControl  # noqa: E402,F401
