"""Coordinator (leader) role + hot-standby mirror.

Reference (worker.py:176-495, 887-1059, 1279-1306): the leader accepts
SUBMIT_JOB_REQUEST (ACK with job id), batches and queues, schedules with the
fair-share/preemption policy, sends WORKER_TASK_REQUEST with image locations,
counts ACKs for C1/C2, tells the requester SUBMIT_JOB_REQUEST_SUCCESS when the
last batch is done, requeues a dead worker's batch at the front and relays
submits/ACKs/file-lists to the H2 standby — which did NOT mirror in-progress
work or batch-size changes, so a takeover re-ran every un-ACKed batch.

Here the standby mirror receives every state transition (submit, dispatch,
preempt, complete, requeue, batch size) plus a periodic full snapshot; on
takeover it adopts running assignments as-is (their workers ACK to the new
leader), and only batches of dead workers are requeued.
"""
from __future__ import annotations

import asyncio
import logging
import time
from typing import Callable, Dict, List, Optional, Tuple

from ..cluster.frames import Frame, MsgType
from ..cluster.membership import MembershipList
from ..cluster.transport import Endpoint
from ..utils import trace as _trace
from .cost_model import CostModel
from .jobs import MODELS, Batch, Job, JobManager
from .journal import JobJournal
from .metrics import Metrics
from .scheduler import plan
from ..cluster.tasks import spawn

log = logging.getLogger(__name__)


class Coordinator:
    def __init__(self, ep: Endpoint, ml: MembershipList, list_images: Callable[[str], List[str]],
                 locate: Callable[[str], Dict[str, List[int]]], batch_sizes: Optional[Dict[str, int]] = None,
                 is_active: Callable[[], bool] = lambda: True, worker_filter: Optional[Callable[[str], bool]] = None,
                 clock=time.monotonic, journal: Optional[JobJournal] = None):
        self.ep, self.ml = ep, ml
        self.list_images = list_images    # pattern -> sorted image names in the store
        self.locate = locate              # image -> {node: [versions]}
        self.jobs = JobManager(batch_sizes)
        self.cost = CostModel()
        self.metrics = Metrics(clock=clock)
        self.running: Dict[str, Tuple[str, tuple, float]] = {}   # worker -> (model, key, t_dispatch)
        self.is_active = is_active
        self.worker_filter = worker_filter or (lambda n: (self.ml.get(n) is not None
                                                          and self.ml.get(n).meta.get("role") == "worker"))
        self.clock = clock
        self.sched_lock = asyncio.Lock()
        self.dispatched = 0
        self.preemptions = 0
        self.requeues = 0
        on = ep.on
        on(MsgType.SUBMIT_JOB_REQUEST, self._on_submit)
        on(MsgType.WORKER_TASK_REQUEST_ACK, self._on_worker_ack)
        on(MsgType.SET_BATCH_SIZE, self._on_set_batch_size)
        on(MsgType.GET_C2_COMMAND, self._on_c2)
        on(MsgType.GET_C1_COMMAND, self._on_c1)
        on(MsgType.GET_ASSIGNMENTS, self._on_assignments)
        on(MsgType.JOB_STATUS, self._on_job_status)
        self.mirror = StandbyMirror(self)
        on(MsgType.STANDBY_SYNC, self.mirror.on_sync)
        self.journal = journal
        self.recovered = self._recover() if journal is not None else 0

    def _recover(self) -> int:
        """Replay the journal (same apply path as the standby mirror); batches
        in flight at the crash go back to the front of their queues."""
        n = self.journal.replay(self.mirror.apply)
        for w in list(self.running):
            self._requeue_worker(w, relay=False)
        if n:
            log.info("coordinator recovered %d journal entries: %d queued batches", n, self.jobs.pending())
            self.journal.compact(self.jobs.snapshot())
        return n

    # ------------------------------------------------------------ helpers --
    def workers(self) -> List[str]:
        return [n for n in self.ml.alive() if self.worker_filter(n)]

    def standbys(self) -> List[str]:
        return [n for n in self.ml.alive(include_self=False)
                if self.ml.get(n).meta.get("role") == "standby"]

    async def relay(self, op: str, **kw) -> None:
        if self.journal is not None:
            self.journal.append(op, **kw)
            self.journal.maybe_compact(self.jobs.snapshot)
        for s in self.standbys():
            await self.ep.send(s, MsgType.STANDBY_SYNC, {"op": op, **kw})

    # ------------------------------------------------------------- submit --
    async def submit(self, model: str, n_images: int, requester: str) -> Job:
        images = self.list_images("*.jpeg")
        job = self.jobs.submit(model, n_images, images, requester, now=self.clock())
        _trace.get_tracer().instant("submit", cat="job", job=job.job_id, model=model, images=n_images,
                                    batches=job.batches_total)
        batches = [b.to_dict() for b in self.jobs.queues[model] if b.job_id == job.job_id]
        await self.relay("submit", job={"job_id": job.job_id, "model": model, "n_images": n_images,
                                        "requester": requester, "batches_total": job.batches_total,
                                        "submitted_at": job.submitted_at}, batches=batches)
        return job

    async def _on_submit(self, fr: Frame) -> None:
        if not self.is_active():
            return
        p = fr.payload
        job = await self.submit(p["model"], int(p["images_count"]), fr.sender)
        await self.ep.reply(fr, MsgType.SUBMIT_JOB_REQUEST_ACK, {"jobid": job.job_id,
                                                                 "batches": job.batches_total})
        if job.batches_total == 0:  # empty store: finished immediately
            await self.ep.send(fr.sender, MsgType.SUBMIT_JOB_REQUEST_SUCCESS, {"jobid": job.job_id})
        await self.schedule()

    # ------------------------------------------------------------ schedule --
    async def schedule(self) -> int:
        if not self.is_active():
            return 0
        async with self.sched_lock:
            online = self.workers()
            # forget assignments of workers that are no longer alive (their batches were requeued)
            for w in [w for w in self.running if w not in online]:
                self._requeue_worker(w)
            free = [w for w in online if w not in self.running]
            queued = {m: len(self.jobs.queues[m]) for m in MODELS}
            assigns = plan(queued, free, {w: (m, k) for w, (m, k, _) in self.running.items()}, online, self.cost,
                           self.jobs.batch_sizes)
            n = 0
            for a in assigns:
                if a.preempt is not None:
                    pm, pkey = a.preempt
                    self.jobs.requeue_front(pkey)
                    self.running.pop(a.worker, None)
                    self.preemptions += 1
                    _trace.get_tracer().end_async("batch", f"{pkey[0]}:{pkey[1]}", cat="job", outcome="preempted")
                    await self.relay("requeue", key=list(pkey))
                b = self.jobs.pop_next(a.model)
                if b is None:
                    continue
                await self._dispatch(a.worker, b)
                n += 1
            return n

    async def _dispatch(self, worker: str, b: Batch) -> None:
        images = {img: self.locate(img) for img in b.images}
        self.running[worker] = (b.model, b.key, self.clock())
        self.dispatched += 1
        _trace.get_tracer().begin_async("batch", f"{b.job_id}:{b.batch_id}", cat="job", worker=worker,
                                        model=b.model, images=len(b.images), attempt=b.attempts)
        await self.relay("dispatch", worker=worker, batch=b.to_dict())
        r = await self.ep.request(worker, MsgType.WORKER_TASK_REQUEST,
                                  {"jobid": b.job_id, "batchid": b.batch_id, "model": b.model, "images": images},
                                  timeout=1.0, retries=2)
        if r is None and not self.ml.is_alive(worker):
            self._requeue_worker(worker)

    def _requeue_worker(self, worker: str, relay: bool = True) -> Optional[Batch]:
        ent = self.running.pop(worker, None)
        if ent is None:
            return None
        self.requeues += 1
        b = self.jobs.requeue_front(ent[1])
        _trace.get_tracer().end_async("batch", f"{ent[1][0]}:{ent[1][1]}", cat="job", outcome="requeued")
        if relay:
            spawn(self.relay("requeue", key=list(ent[1])))
        return b

    def worker_failed(self, worker: str) -> None:
        """Membership callback (reference handle_failures_if_pending_status, worker.py:1279-1306)."""
        if self._requeue_worker(worker) is not None:
            log.info("requeued batch of failed worker %s", worker)
        if self.is_active():
            spawn(self.schedule())

    # ---------------------------------------------------------------- acks --
    async def _on_worker_ack(self, fr: Frame) -> None:
        await self.ep.reply(fr, MsgType.ACK, {})
        if not self.is_active():
            return
        p = fr.payload
        key = (int(p["jobid"]), int(p["batchid"]))
        ent = self.running.get(fr.sender)
        if ent is not None and ent[1] == key:
            del self.running[fr.sender]
            latency = self.clock() - ent[2]
        else:
            latency = float(p.get("service_time", 0.0))
        job = self.jobs.complete(key, now=self.clock())
        if job is not None:
            n = int(p.get("image_count", 0))
            _trace.get_tracer().end_async("batch", f"{key[0]}:{key[1]}", cat="job", outcome="done",
                                          latency_ms=latency * 1e3)
            self.metrics.record(p["model"], latency, float(p.get("service_time", latency)), n)
            self.cost.observe(p["model"], n, float(p.get("service_time", latency)))
            await self.relay("complete", key=list(key), model=p["model"], latency=latency,
                             service=float(p.get("service_time", latency)), images=n)
            if job.done:
                await self.ep.send(job.requester, MsgType.SUBMIT_JOB_REQUEST_SUCCESS, {"jobid": job.job_id})
        await self.schedule()

    # ------------------------------------------------------------ commands --
    async def _on_set_batch_size(self, fr: Frame) -> None:
        m, bs = fr.payload["model"], int(fr.payload["batch_size"])
        self.jobs.set_batch_size(m, bs)   # per-model (reference always used Inception's timing, worker.py:1035)
        await self.relay("batch_size", model=m, batch_size=bs)
        if fr.seq:
            await self.ep.reply(fr, MsgType.SET_BATCH_SIZE_ACK, {"model": m, "batch_size": bs})

    async def _on_c2(self, fr: Frame) -> None:
        p = self.metrics.c2_reference_payload()
        p["detail"] = self.metrics.c2()
        await self.ep.reply(fr, MsgType.GET_C2_COMMAND_ACK, p)

    async def _on_c1(self, fr: Frame) -> None:
        await self.ep.reply(fr, MsgType.GET_C1_COMMAND_ACK, {"c1": self.metrics.c1()})

    def assignments(self) -> Dict[str, dict]:
        """C5: {worker: {model, job_id, batch_id}} (reference workers_tasks_dict)."""
        return {w: {"model": m, "job_id": k[0], "batch_id": k[1]} for w, (m, k, _) in sorted(self.running.items())}

    async def _on_assignments(self, fr: Frame) -> None:
        await self.ep.reply(fr, MsgType.GET_ASSIGNMENTS_ACK, {"assignments": self.assignments()})

    async def _on_job_status(self, fr: Frame) -> None:
        j = self.jobs.jobs.get(int(fr.payload["jobid"]))
        await self.ep.reply(fr, MsgType.JOB_STATUS_ACK,
                            {"jobid": fr.payload["jobid"], "known": j is not None,
                             "done": bool(j and j.done), "batches_done": j.batches_done if j else 0,
                             "batches_total": j.batches_total if j else 0})

    # ------------------------------------------------------------ takeover --
    def take_over(self) -> None:
        """Standby became leader: requeue only batches whose worker is gone."""
        for w in [w for w in self.running if not self.ml.is_alive(w)]:
            self._requeue_worker(w)


class StandbyMirror:
    """Applies the active coordinator's relayed transitions to the local state."""

    def __init__(self, coord: Coordinator):
        self.c = coord
        self.applied = 0

    async def on_sync(self, fr: Frame) -> None:
        if self.c.is_active():
            return
        self.apply(fr.payload)

    def apply(self, p: dict) -> None:
        """Apply one relayed / journaled transition to the local state."""
        c = self.c
        op = p.get("op")
        jm = c.jobs
        if op == "snapshot":
            jm.restore(p["state"], requeue_inprogress=True)
            c.running.clear()
        elif op == "submit":
            j = p["job"]
            jm.jobs[j["job_id"]] = Job(j["job_id"], j["model"], j["n_images"], j["requester"], j["batches_total"],
                                       0, j.get("submitted_at", 0.0))
            jm.queues[j["model"]].extend(Batch.from_dict(b) for b in p["batches"])
            import itertools

            jm._ids = itertools.count(max(jm.jobs) + 1)
        elif op == "dispatch":
            b = Batch.from_dict(p["batch"])
            q = jm.queues[b.model]
            for i, x in enumerate(q):
                if x.key == b.key:
                    del q[i]
                    break
            jm.inprogress[b.key] = b
            c.running[p["worker"]] = (b.model, b.key, c.clock())
        elif op == "requeue":
            key = tuple(p["key"])
            for w, (m, k, _) in list(c.running.items()):
                if k == key:
                    del c.running[w]
            jm.requeue_front(key)
        elif op == "complete":
            key = tuple(p["key"])
            for w, (m, k, _) in list(c.running.items()):
                if k == key:
                    del c.running[w]
            if jm.complete(key) is not None:
                c.metrics.record(p["model"], p["latency"], p["service"], p["images"])
        elif op == "batch_size":
            jm.set_batch_size(p["model"], int(p["batch_size"]))
        self.applied += 1
