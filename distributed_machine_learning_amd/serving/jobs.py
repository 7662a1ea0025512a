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
from typing import Deque, Dict, List, Optional, Sequence

MODELS = ("ResNet50", "InceptionV3")
FIRST_JOB_ID = 31
SYNTH = "synthetic:"


class SynthNames(Sequence):
    """The synthetic image names SYNTH + str(i) for i in [lo, hi), never materialised: a
    9,600-batch synthetic job is two integers in the replicated log and per batch, not 2.4M
    strings JSON-encoded, broadcast and rebuilt on every rank in one step (measured: a 200 ms
    stall of the whole lockstep group at world 8, tools/store_capacity.py)."""

    __slots__ = ("lo", "hi")

    def __init__(self, lo: int, hi: int):
        self.lo, self.hi = int(lo), max(int(lo), int(hi))

    def __len__(self) -> int:
        return self.hi - self.lo

    def __getitem__(self, i):
        if isinstance(i, slice):
            a, b, st = i.indices(len(self))
            if st == 1:
                return SynthNames(self.lo + a, self.lo + max(a, b))
            return [self[j] for j in range(a, b, st)]
        n = len(self)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError(i)
        return f"{SYNTH}{self.lo + i}"

    def __iter__(self):
        return (f"{SYNTH}{i}" for i in range(self.lo, self.hi))

    def __eq__(self, other) -> bool:
        if isinstance(other, SynthNames):
            return (self.lo, self.hi) == (other.lo, other.hi) or (len(self) == 0 and len(other) == 0)
        try:
            return len(other) == len(self) and all(a == b for a, b in zip(self, other))
        except TypeError:
            return NotImplemented

    def __hash__(self):
        return hash((self.lo, self.hi))

    def __repr__(self) -> str:
        return f"SynthNames({self.lo}, {self.hi})"

    def to_json(self) -> dict:
        return {"synth": [self.lo, self.hi]}


def as_names(x) -> Sequence[str]:
    """An image list from a log record / snapshot: SynthNames stay lazy ({"synth": [lo, hi]} in
    JSON), anything else becomes a list."""
    if isinstance(x, SynthNames):
        return x
    if isinstance(x, dict) and "synth" in x:
        return SynthNames(*x["synth"])
    return list(x)


def json_default(o):
    """json.dumps(default=...) for records that carry SynthNames."""
    if isinstance(o, SynthNames):
        return o.to_json()
    raise TypeError(f"not JSON serializable: {type(o).__name__}")


@dataclass
class Batch:
    job_id: int
    batch_id: int
    model: str
    images: Sequence[str]      # a list, or SynthNames (lazy synthetic names)
    attempts: int = 0          # dispatches so far (preemption / failure re-dispatch)

    @property
    def key(self):
        return (self.job_id, self.batch_id)

    def to_dict(self) -> dict:
        return {"job_id": self.job_id, "batch_id": self.batch_id, "model": self.model,
                "images": self.images.to_json() if isinstance(self.images, SynthNames) else list(self.images),
                "attempts": self.attempts}

    @staticmethod
    def from_dict(d: dict) -> "Batch":
        return Batch(int(d["job_id"]), int(d["batch_id"]), d["model"], as_names(d["images"]), int(d.get("attempts", 0)))


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


def make_batches(job_id: int, model: str, images: Sequence[str], batch_size: int) -> List[Batch]:
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
        images = as_names(images)
        batches = make_batches(jid, model, images, self.batch_sizes[model])
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
