"""Job intake and batching (coordinator side).

Reference (worker.py:176-245, 911-920): job ids are a counter initialised to 30
(first job = 31); N images are picked CYCLICALLY from the sorted ``*.jpeg``
list of the store; they are cut into batches with ids 1..B and appended to the
model's FIFO queue; the requester is remembered with a pending-batch count.
Defect fixed: the reference's batches hold ``batch_size + 1`` images (100 at
bs=10 gave [11 x 9, 1]); here every batch holds exactly ``batch_size``.
"""
from __future__ import annotations

import itertools
from collections import deque
from dataclasses import asdict, dataclass
from typing import Deque, Dict, List, Optional

MODELS = ("ResNet50", "InceptionV3")
FIRST_JOB_ID = 31


@dataclass
class Batch:
    job_id: int
    batch_id: int
    model: str
    images: List[str]
    attempts: int = 0          # dispatches so far (preemption / failure re-dispatch)

    @property
    def key(self):
        return (self.job_id, self.batch_id)

    def to_dict(self) -> dict:
        return asdict(self)

    @staticmethod
    def from_dict(d: dict) -> "Batch":
        return Batch(int(d["job_id"]), int(d["batch_id"]), d["model"], list(d["images"]), int(d.get("attempts", 0)))


@dataclass
class Job:
    job_id: int
    model: str
    n_images: int
    requester: str
    batches_total: int = 0
    batches_done: int = 0
    submitted_at: float = 0.0
    finished_at: Optional[float] = None

    @property
    def done(self) -> bool:
        return self.batches_total > 0 and self.batches_done >= self.batches_total


def pick_images(sorted_images: List[str], n: int) -> List[str]:
    """Cyclic selection from the sorted store listing (worker.py:196-206)."""
    if not sorted_images:
        return []
    return [sorted_images[i % len(sorted_images)] for i in range(n)]


def make_batches(job_id: int, model: str, images: List[str], batch_size: int) -> List[Batch]:
    if batch_size < 1:
        raise ValueError("batch_size must be >= 1")
    return [Batch(job_id, i // batch_size + 1, model, images[i:i + batch_size])
            for i in range(0, len(images), batch_size)]


class JobManager:
    def __init__(self, batch_sizes: Optional[Dict[str, int]] = None, first_job_id: int = FIRST_JOB_ID):
        self._ids = itertools.count(first_job_id)
        self.jobs: Dict[int, Job] = {}
        self.queues: Dict[str, Deque[Batch]] = {m: deque() for m in MODELS}
        self.inprogress: Dict[tuple, Batch] = {}
        self.batch_sizes = dict(batch_sizes or {m: 10 for m in MODELS})

    def next_id(self) -> int:
        return next(self._ids)

    def submit(self, model: str, n_images: int, store_images: List[str], requester: str, now: float = 0.0,
               job_id: Optional[int] = None) -> Job:
        if model not in self.queues:
            raise KeyError(f"unknown model {model}")
        jid = job_id if job_id is not None else self.next_id()
        images = pick_images(sorted(store_images), n_images)
        batches = make_batches(jid, model, images, self.batch_sizes[model])
        job = Job(jid, model, n_images, requester, len(batches), 0, now)
        self.jobs[jid] = job
        self.queues[model].extend(batches)
        return job

    def submit_images(self, model: str, images: List[str], requester: str, now: float = 0.0,
                      job_id: Optional[int] = None) -> Job:
        """Submit an explicit image list (already selected) as one job. An
        explicit ``job_id`` (a replicated log record) also advances the counter."""
        if model not in self.queues:
            raise KeyError(f"unknown model {model}")
        if job_id is None:
            jid = self.next_id()
        else:
            jid = int(job_id)
            self._ids = itertools.count(max([jid] + list(self.jobs)) + 1)
        batches = make_batches(jid, model, list(images), self.batch_sizes[model])
        job = Job(jid, model, len(images), requester, len(batches), 0, now)
        self.jobs[jid] = job
        self.queues[model].extend(batches)
        return job

    def set_batch_size(self, model: str, bs: int) -> None:
        if bs < 1:
            raise ValueError("batch size must be >= 1")
        self.batch_sizes[model] = bs

    def pop_next(self, model: str) -> Optional[Batch]:
        q = self.queues[model]
        if not q:
            return None
        b = q.popleft()
        b.attempts += 1
        self.inprogress[b.key] = b
        return b

    def pop_key(self, model: str, key: tuple) -> Optional[Batch]:
        """Take a specific queued batch (a replica applying the coordinator's dispatch)."""
        q = self.queues[model]
        for i, b in enumerate(q):
            if b.key == key:
                del q[i]
                b.attempts += 1
                self.inprogress[b.key] = b
                return b
        return None

    def requeue_front(self, key: tuple) -> Optional[Batch]:
        """Preempted or failed batch goes back to the FRONT of its queue (worker.py:406-408, 1284-1306)."""
        b = self.inprogress.pop(key, None)
        if b is not None:
            self.queues[b.model].appendleft(b)
        return b

    def complete(self, key: tuple, now: float = 0.0) -> Optional[Job]:
        b = self.inprogress.pop(key, None)
        if b is None:
            return None  # duplicate / stale ACK (at-least-once delivery after takeover)
        job = self.jobs.get(b.job_id)
        if job is not None:
            job.batches_done += 1
            if job.done and job.finished_at is None:
                job.finished_at = now
        return job

    def pending(self, model: Optional[str] = None) -> int:
        ms = [model] if model else list(self.queues)
        return sum(len(self.queues[m]) for m in ms)

    # -------- standby mirroring (full state, incl. in-progress: the reference
    # -------- did not mirror inprogress_queue, worker.py:887-897, 965-985)
    def snapshot(self) -> dict:
        return {"queues": {m: [b.to_dict() for b in q] for m, q in self.queues.items()},
                "inprogress": [b.to_dict() for b in self.inprogress.values()],
                "jobs": {j: asdict(v) for j, v in self.jobs.items()},
                "batch_sizes": self.batch_sizes}

    def restore(self, snap: dict, requeue_inprogress: bool = True) -> None:
        self.queues = {m: deque(Batch.from_dict(d) for d in snap["queues"].get(m, [])) for m in MODELS}
        self.jobs = {int(k): Job(**v) for k, v in snap["jobs"].items()}
        self.batch_sizes.update(snap.get("batch_sizes", {}))
        inprog = [Batch.from_dict(d) for d in snap.get("inprogress", [])]
        self.inprogress = {}
        if requeue_inprogress:
            for b in reversed(inprog):
                self.queues[b.model].appendleft(b)
        else:
            self.inprogress = {b.key: b for b in inprog}
        if self.jobs:
            self._ids = itertools.count(max(self.jobs) + 1)
