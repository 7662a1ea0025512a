"""Elastic multi-GPU serving: one process per GPU, RCCL data plane, a
REPLICATED coordinator, SWIM liveness, the reference's CLI and store.

Reference: the leader (H1) owns all job state and relays submits/ACKs to one
hard-coded standby (H2) over UDP (worker.py:176-495, 887-1037, 577-614); if both
die nothing can take over (election.py:27). Here every rank holds the whole
coordinator state as a replicated state machine driven by the step's
collectives, so ANY survivor can continue as coordinator:

  step k (every rank; steps run at host speed, independent of GPU progress):
    coordinator  drains its control inbox (client submits / C3 from the CLI) into
                 log records, applies them, plans step k's dispatch table: at most
                 one new batch for each rank whose work queue holds fewer than
                 ``depth`` (2) batches, fair-share between the two models
    broadcast    header [log length, step, table] from the coordinator (48 B per
                 rank), then the log payload (JSON) if any
    every rank   applies the same log records and the same table -> identical
                 queues, in-flight sets and job-id counters on every rank, and
                 enqueues its own new batch on its GPU (arena slots -> H2D ->
                 hipGraph forward; the queue keeps the GPU busy)
    all-gather   at most one COMPLETED batch per rank (its GPU event polled,
                 never waited on): packed top-5 [2, cap, 5] int32 + batch key ->
                 every rank completes those batches identically (C1 counts, job
                 completion); the coordinator also writes
                 output_<job>_<batch>_<host>.json and PUTs it into the store
  No rank ever waits for another rank's compute: a ResNet50 rank and an
  InceptionV3 rank run their own queues (the old lockstep step cost the slowest
  rank's batch time on every rank).

  These step collectives carry control-sized messages (48 B per rank + 10 KB of
  packed top-5), so they run on a host (gloo) group by default: issued as RCCL
  kernels they queue behind the forward's kernels on the GPU, and a step then
  waits for a whole batch (1 GPU, concurrent ResNet50 + InceptionV3: 41.0k
  img/s over RCCL vs 61.5k over gloo = 98 % of the time-weighted single-model
  rates; profiles/r2_v3). The ``nccl`` backend stays supported (GPU-tested).

  The coordinator is the highest alive global rank — the same rank the
  control plane's bully election (cluster/election.py, prio = rank) makes the
  store leader, so the CLI's leader requests reach it.

Failure: SWIM (host UDP, never RCCL) confirms a dead rank -> pending collectives
are aborted (parallel/elastic.py) -> every survivor requeues all in-flight
batches at the FRONT of their queues (identical replicas, so identical result)
-> the communicator is rebuilt over the survivors (FileStore rendezvous: no rank
hosts it) -> the new coordinator broadcasts its full job state (repairs any
replica that completed one step more or less than it did) and re-PUTs the output
files of the last completed steps (a dead coordinator may not have written them:
at-least-once outputs). Batches may run twice; every job completes.

Images: a job names store images (cyclic pick over the sorted ``*.jpeg``
listing, reference worker.py:176-206) or synthetic images. Applying a submit
record, every rank fetches and decodes only ITS SHARE of the job's new images
and one all-gather over the data group (RCCL over xGMI) replicates the decoded
tensors into every rank's HBM image store (parallel/image_store.py): each
image is decoded once per job, not once per rank. A batch is a list of store
slots gathered on the GPU. C3 (per-model batch size) is a replicated log
record, clamped to the result capacity; a batch larger than the engine's batch
runs as several engine passes (never truncated).
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import queue
import threading
import time
from collections import OrderedDict, deque
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..serving.cost_model import CostModel
from ..serving.jobs import MODELS, Batch, JobManager
from ..serving.metrics import Metrics
from ..serving.output import decode_top5, dumps, output_name
from ..serving.scheduler import plan
from .dataplane import DESC_FIELDS, F_BATCH, F_JOB, F_MODEL
from .elastic import CollectiveFailure, ElasticGroup

log = logging.getLogger(__name__)
MODEL_IDS = {m: i for i, m in enumerate(MODELS)}
IDLE, STOP = -1, -2
SYNTH = "synthetic:"          # synthetic arena image names: "synthetic:<index>"
HDR = 3                       # header words before the table: log length, step, flags
RESULT_HISTORY = 64           # completed steps whose results every rank keeps (output re-PUT on takeover)


def synthetic_names(n: int) -> List[str]:
    return [f"{SYNTH}{i}" for i in range(n)]


# --------------------------------------------------------------- backends ----
class RankBackend:
    """Runs one batch (a list of image names) of ``model`` on this rank.

    ``launch`` is asynchronous on GPU backends: it enqueues staging + forward and
    returns (result [2, cap, 5] int32, completion event or None) — rows of
    images that could not be fetched or decoded carry class id -1 — so the
    service gathers the previous step's results while this batch runs.
    ``cap`` (result rows) bounds the batch size the coordinator may assign."""

    cap: int = 256
    device = torch.device("cpu")

    def launch(self, model: str, names: Sequence[str], slot: int):
        raise NotImplementedError

    def run(self, model: str, names: Sequence[str]) -> torch.Tensor:
        res, ev = self.launch(model, names, 0)
        if ev is not None:
            ev.synchronize()
        return res


class HostRankBackend(RankBackend):
    """A serving.inference backend (fake / cpu) behind the rank interface:
    decode-once per image name (LRU cache), synchronous predict. The same
    backend classes as the host cluster's workers, so both serving modes produce
    identical outputs for the same images. Synthetic names decode from their own
    name bytes; failed images get class id -1 in their result row."""

    def __init__(self, backend, loader: Optional[Callable] = None, cap: int = 256, delay_per_image: float = 0.0,
                 cache_images: int = 4096):
        self.be, self.loader, self.cap, self.delay = backend, loader, cap, delay_per_image
        self.cache: "OrderedDict[Tuple[str, str], np.ndarray]" = OrderedDict()
        self.cache_images = cache_images

    def _blobs(self, names: List[str]) -> Dict[str, Optional[bytes]]:
        out = {n: n.encode() for n in names if n.startswith(SYNTH)}
        rest = [n for n in names if not n.startswith(SYNTH)]
        if rest:
            out.update(self.loader(rest) if self.loader else {n: None for n in rest})
        return out

    def launch(self, model, names, slot):
        if len(names) > self.cap:
            raise ValueError(f"batch of {len(names)} exceeds the result capacity {self.cap}")
        if self.delay:
            time.sleep(self.delay * len(names))
        missing = [n for n in dict.fromkeys(names) if (model, n) not in self.cache]
        failed = set()
        if missing:
            blobs = self._blobs(missing)
            for n in missing:
                b = blobs.get(n)
                try:
                    self.cache[(model, n)] = self.be.decode_batch(model, [b])[0] if b is not None else None
                except Exception as e:
                    log.warning("decode of %s failed: %s", n, e)
                    self.cache[(model, n)] = None
            while len(self.cache) > self.cache_images:
                self.cache.popitem(last=False)
        imgs = []
        for n in names:
            im = self.cache.get((model, n))
            if im is None:
                failed.add(n)
            else:
                self.cache.move_to_end((model, n))
                imgs.append(im)
        out = torch.zeros((2, self.cap, 5), dtype=torch.int32)
        ok = [i for i, n in enumerate(names) if n not in failed]
        if ok:
            idx, p = self.be.predict(model, np.stack(imgs))
            rows = torch.tensor(ok, dtype=torch.long)
            out[0, rows] = torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int32))
            out[1, rows] = torch.from_numpy(np.ascontiguousarray(p, dtype=np.float32)).view(torch.int32)
        for i, n in enumerate(names):
            if n in failed:
                out[0, i] = -1
        return out, None


class FakeRankBackend(HostRankBackend):
    """Deterministic pseudo-results (serving.inference.FakeBackend), optional
    per-image delay (CPU tests)."""

    def __init__(self, cap: int = 16, delay_per_image: float = 0.0, loader: Optional[Callable] = None):
        from ..serving.inference import FakeBackend

        super().__init__(FakeBackend(), loader=loader, cap=cap, delay_per_image=delay_per_image)


class GpuRankBackend(RankBackend):
    """Native engines for both models resident in this GPU's HBM, fed from
    per-model HBM image stores (parallel/image_store.py: store images decoded
    once per job and replicated to every rank over the data group — RCCL —
    plus seeded synthetic images). A batch is gathered from the store into the
    engine's source slot on the compute stream, in order (no PCIe copy per
    batch, nothing for another queue to starve); results land in one of two
    output slots. A batch larger than the engine's batch runs as several engine
    passes into consecutive result rows."""

    def __init__(self, device: torch.device, batch_sizes: Dict[str, int], cap: int = 0, arena_images: int = 8192,
                 n_synth: int = 512, seed: int = 0, models: Sequence[str] = MODELS, splits: int = 2,
                 loader: Optional[Callable] = None, decode_threads: int = 8):
        from concurrent.futures import ThreadPoolExecutor

        from ..models import build_model
        from ..models.engine import Engine, SplitEngine
        from .image_store import HbmImageStore

        self.device = device
        self.cap = cap or max(batch_sizes.values())
        self.loader = loader
        self.engines, self.arenas = {}, {}
        self.stream = torch.cuda.Stream(device)
        self.pool = ThreadPoolExecutor(max_workers=decode_threads)
        for m in models:
            g, w = build_model(m, seed=seed, calibrate=True)
            b = batch_sizes[m]
            if splits > 1 and b % splits == 0:
                self.engines[m] = SplitEngine(g, w, batch=b, device=str(device), src_slots=2, splits=splits)
            else:
                self.engines[m] = Engine(g, w, batch=b, device=str(device), src_slots=2)
            self.arenas[m] = HbmImageStore(max(arena_images, n_synth + 2 * self.cap), g.input_hw, device,
                                           n_synth=n_synth, seed=1000 + MODEL_IDS[m])
            self.engines[m].capture(self.stream)  # graphs now, before the service's first collective
        self.out = [torch.zeros((2, self.cap, 5), dtype=torch.int32, device=device) for _ in range(2)]
        self.ev_done = [torch.cuda.Event() for _ in range(2)]

    def _load(self, model: str, names: List[str]) -> Dict[str, Optional[np.ndarray]]:
        from ..serving.inference import load_image

        blobs = self.loader(names) if self.loader else {}
        hw = self.arenas[model].hw

        def dec(n):
            b = blobs.get(n)
            if b is None:
                return n, None
            try:
                return n, load_image(b, hw)
            except Exception as e:  # undecodable file -> reported as failed
                log.warning("decode of %s failed: %s", n, e)
                return n, None
        return dict(self.pool.map(dec, names))

    def on_submit(self, model: str, names: Sequence[str], eg: ElasticGroup) -> int:
        """(collective, every rank) decode this rank's share of the job's new
        images and all-gather all shares into every rank's HBM store."""
        n = self.arenas[model].replicate(names, lambda ns: self._load(model, ns), rank=eg.rank, world=eg.world,
                                         gather=eg.all_gather_data)
        torch.cuda.current_stream(self.device).synchronize()  # store writes visible to the compute stream
        return n

    def launch(self, model, names, slot):
        if len(names) > self.cap:
            raise ValueError(f"batch of {len(names)} exceeds the result capacity {self.cap}")
        eng, arena = self.engines[model], self.arenas[model]
        slots, failed = arena.slots(list(names), lambda ns: self._load(model, ns))
        s = self.stream
        out = self.out[slot]
        B = eng.batch
        with torch.cuda.stream(s):
            for off in range(0, len(slots), B):  # one engine pass per B images: never truncated
                chunk = slots[off:off + B]
                arena.gather_into(eng.srcs[slot], chunk)
                eng.run(s, use_graph=True, slot=slot)
                out[:, off:off + len(chunk)].copy_(eng.results[slot][:, :len(chunk)])
            if failed:  # unfetchable / undecodable images: class id -1 marks the row failed
                bad = set(failed)
                rows = torch.tensor([i for i, n in enumerate(names) if n in bad], dtype=torch.long)
                out[0].index_fill_(0, rows.pin_memory().to(self.device, non_blocking=True), -1)
            self.ev_done[slot].record(s)
        return out, self.ev_done[slot]


# ------------------------------------------------------------- coordinator ----
@dataclass
class Inflight:
    rank: int
    batch: Batch
    t_dispatch: float
    seq: int            # dispatch order (requeue restores queue order)


class ReplicatedCoordinator:
    """The job service's state machine (reference leader, worker.py:176-495,
    989-1037), identical on every rank: log records and dispatch tables are
    applied in broadcast order, completions in all-gather order. Only the active
    coordinator PLANS tables (its cost model is timing-dependent) and writes
    outputs; replicas apply what it broadcast. Each rank may hold up to
    ``depth`` dispatched batches (its GPU work queue)."""

    def __init__(self, batch_sizes: Dict[str, int], cap: int = 256, host_tag: str = "node", depth: int = 2):
        self.cap, self.depth = cap, depth
        self.jobs = JobManager({m: min(int(b), cap) for m, b in batch_sizes.items()})
        self.cost = CostModel()
        self.metrics = Metrics()
        self.inflight: "OrderedDict[tuple, Inflight]" = OrderedDict()   # batch key -> assignment
        self.seq = 0
        self.requeued = 0
        self.host_tag = host_tag
        self.lock = threading.RLock()      # control-thread readers (C1/C2/C5/status) vs the serve loop
        self.history: "OrderedDict[tuple, tuple]" = OrderedDict()  # key -> (batch, idx, p, grank), recent

    # ------------------------------------------------------------- log ----
    def apply(self, rec: dict) -> dict:
        """Apply one replicated log record; returns what the requester is told."""
        op = rec["op"]
        if op == "submit":
            jm = self.jobs
            job = jm.submit_images(rec["model"], list(rec["images"]), rec.get("requester", "client"),
                                   now=time.monotonic(), job_id=int(rec["job_id"]))
            return {"jobid": job.job_id, "batches": job.batches_total}
        if op == "batch_size":
            bs = max(1, min(int(rec["batch_size"]), self.cap))
            self.jobs.set_batch_size(rec["model"], bs)
            return {"model": rec["model"], "batch_size": bs}
        if op == "state":  # new coordinator's full state after a rebuild
            self.jobs.restore(rec["jobs"], requeue_inprogress=True)
            self.inflight.clear()
            return {}
        raise ValueError(f"unknown log record {op}")

    def next_job_id(self, pending: int = 0) -> int:
        """Id the next submit will get once applied (records apply in order)."""
        return max([30] + list(self.jobs.jobs)) + 1 + pending

    def idle(self) -> bool:
        return self.jobs.pending() == 0 and not self.jobs.inprogress

    def outstanding(self, grank: int) -> int:
        return sum(1 for inf in self.inflight.values() if inf.rank == grank)

    # ---------------------------------------------------------- tables ----
    def next_table(self, members: List[int]) -> np.ndarray:
        """(active coordinator) at most one new batch per rank whose queue has
        room: fair-share split of those ranks between the two models' queues
        (reference worker.py:255-495)."""
        t = np.zeros((len(members), DESC_FIELDS), np.int64)
        t[:, F_MODEL] = IDLE
        queued = {m: len(self.jobs.queues[m]) for m in MODELS}
        free = [g for g in members if self.outstanding(g) < self.depth]
        if not any(queued.values()) or not free:
            return t
        workers = [f"rank{g}" for g in free]
        online = [f"rank{g}" for g in members]
        running = {}
        for inf in self.inflight.values():  # what every rank is busy with (fair-share input)
            running.setdefault(f"rank{inf.rank}", (inf.batch.model, inf.batch.key))
        running = {w: v for w, v in running.items() if w not in workers}
        assigns = plan(queued, workers, running, online, self.cost, self.jobs.batch_sizes, preempt=False)
        taken = {m: 0 for m in MODELS}
        for a in assigns:
            q = self.jobs.queues[a.model]
            if taken[a.model] >= len(q):
                continue
            b = q[taken[a.model]]   # popped for real by apply_table, on every rank
            taken[a.model] += 1
            g = int(a.worker[4:])
            t[members.index(g)] = (b.job_id, b.batch_id, MODEL_IDS[b.model], 0, len(b.images), 0)
        return t

    def apply_table(self, table: np.ndarray, members: List[int]) -> None:
        """Take exactly the broadcast batches out of the local queues (every
        rank, the coordinator included)."""
        now = time.monotonic()
        for r, g in enumerate(members):
            if int(table[r, F_MODEL]) < 0:
                continue
            model = MODELS[int(table[r, F_MODEL])]
            b = self.jobs.pop_key(model, (int(table[r, F_JOB]), int(table[r, F_BATCH])))
            if b is None:
                raise RuntimeError(f"replica diverged: batch {table[r, F_JOB]}:{table[r, F_BATCH]} not queued")
            self.inflight[b.key] = Inflight(g, b, now, self.seq)
            self.seq += 1

    def assigned(self, table: np.ndarray, members: List[int], grank: int) -> Optional[Batch]:
        row = table[members.index(grank)]
        if int(row[F_MODEL]) < 0:
            return None
        inf = self.inflight.get((int(row[F_JOB]), int(row[F_BATCH])))
        return None if inf is None else inf.batch

    # -------------------------------------------------------- complete ----
    def complete(self, key: tuple, rows: Optional[np.ndarray], service: float = 0.0
                 ) -> Optional[Tuple[Batch, np.ndarray, np.ndarray, int]]:
        """Batch ``key`` finished (its all-gathered result rows). Returns what
        the output writer needs, or None for an unknown / duplicate key."""
        inf = self.inflight.pop(key, None)
        now = time.monotonic()
        if inf is None or self.jobs.complete(key, now=now) is None:
            return None
        b = inf.batch
        n = len(b.images)
        self.metrics.record(b.model, now - inf.t_dispatch, service or now - inf.t_dispatch, n)
        self.cost.observe(b.model, n, service or now - inf.t_dispatch)
        if rows is None:
            return None
        done = (b, rows[0, :n].copy(), rows[1, :n].view(np.float32).copy(), inf.rank)
        self.history[key] = done
        while len(self.history) > RESULT_HISTORY:
            self.history.popitem(last=False)
        return done

    def requeue_inflight(self) -> int:
        """Failure: every dispatched batch goes back to the FRONT of its queue
        (newest dispatch first, so queue order is preserved)."""
        n = 0
        for inf in sorted(self.inflight.values(), key=lambda i: -i.seq):
            if self.jobs.requeue_front(inf.batch.key) is not None:
                n += 1
        self.inflight.clear()
        self.requeued += n
        return n

    def assignments(self) -> Dict[str, dict]:
        """C5: {rank: {model, job_id, batch_id}} — the oldest batch of each rank's queue."""
        out = {}
        for inf in self.inflight.values():
            out.setdefault(f"rank{inf.rank}", {"model": inf.batch.model, "job_id": inf.batch.job_id,
                                               "batch_id": inf.batch.batch_id})
        return out


# ---------------------------------------------------------- output writer ----
class OutputWriter:
    """Writes output_<job>_<batch>_<host>.json off the serve loop (a blocking
    queue: a file is never dropped) into ``out_dir`` and/or the store."""

    def __init__(self, out_dir: Optional[str], put: Optional[Callable[[str, bytes], None]] = None,
                 host_tag: str = "node"):
        self.out_dir, self.put, self.host_tag = out_dir, put, host_tag
        if out_dir:
            os.makedirs(out_dir, exist_ok=True)
        self.q: "queue.Queue" = queue.Queue()
        self.written = 0
        self.thread = threading.Thread(target=self._loop, daemon=True, name="output-writer")
        self.thread.start()

    def submit(self, b: Batch, idx: np.ndarray, p: np.ndarray, grank: int,
               on_written: Optional[Callable[[Batch], None]] = None) -> None:
        self.q.put((b, idx, p, grank, on_written))

    def _loop(self) -> None:
        while True:
            item = self.q.get()
            if item is None:
                return
            b, idx, p, g, on_written = item
            try:
                failed = [n for i, n in enumerate(b.images) if idx[i, 0] < 0]
                ok = [i for i in range(len(b.images)) if idx[i, 0] >= 0]
                names = [b.images[i] for i in ok]
                doc = decode_top5(names, idx[ok], p[ok], failed)
                name = output_name(b.job_id, b.batch_id, f"{self.host_tag}-rank{g}")
                text = dumps(doc)
                if self.out_dir:
                    with open(os.path.join(self.out_dir, name), "w") as f:
                        f.write(text)
                if self.put is not None:
                    self.put(name, text.encode())
                self.written += 1
                if on_written is not None:
                    on_written(b)
            except Exception as e:  # a failed write is logged, never silently skipped
                log.error("output %s:%s not written: %s", b.job_id, b.batch_id, e)

    def flush(self) -> None:
        """Block until every queued file is written (sentinel + join), then restart."""
        self.q.put(None)
        self.thread.join()
        self.thread = threading.Thread(target=self._loop, daemon=True, name="output-writer")
        self.thread.start()


# ---------------------------------------------------------------- service ----
class CollectiveService:
    """The per-rank serve loop (identical on every rank). See the module doc.

    Per-rank work queues, no lockstep on compute: a step is one broadcast (log
    + dispatch table: at most one new batch per rank whose queue holds fewer
    than ``coord.depth`` batches) and one all-gather of at most one COMPLETED
    batch per rank (a rank contributes a batch once its GPU event has fired —
    polled, never waited on), so the collectives run at host speed while every
    GPU works through its own queue; a ResNet50 rank and an InceptionV3 rank
    never wait for each other. Collectives run on their own HIP stream.

    ``control``: optional RankControl (UDP control plane + store of this rank);
    without it (tests, benches) jobs are submitted with ``submit_local`` on the
    coordinator rank."""

    def __init__(self, eg: ElasticGroup, backend: RankBackend, coord: ReplicatedCoordinator,
                 control=None, writer: Optional[OutputWriter] = None, kill_rank: int = -1, kill_at_step: int = -1,
                 on_device: bool = False, idle_sleep: float = 0.002, poll_sleep: float = 0.0001,
                 watchdog_s: float = 0.0):
        if coord.depth > 2:
            raise ValueError("rank queues deeper than the backends' 2 source/result slots")
        self.eg, self.be, self.coord, self.control = eg, backend, coord, control
        self.writer = writer
        self.kill_rank, self.kill_at_step = kill_rank, kill_at_step
        self.dev = backend.device if on_device else torch.device("cpu")
        self.comm = torch.cuda.Stream(self.dev) if self.dev.type == "cuda" else None
        self.steps = 0
        self.rebuilds = 0
        self.cap = backend.cap
        self.local: "deque" = deque()   # (key, result, event) launched here, not yet reported
        self.launched = 0
        self.sbuf = torch.zeros((2, self.cap + 1, 5), dtype=torch.int32, device=self.dev)
        self.idle_sleep, self.poll_sleep = idle_sleep, poll_sleep
        self._inbox: "queue.Queue" = queue.Queue()   # (record, reply callback or None)
        self._written: Dict[int, set] = {}             # job id -> batch ids whose output is durable
        self._stop = False
        self.last_progress = time.monotonic()
        self.phase_s: Dict[str, float] = {"plan": 0.0, "broadcast": 0.0, "launch": 0.0, "exchange": 0.0,
                                          "complete": 0.0, "sleep": 0.0}
        self._watchdog = None
        if watchdog_s > 0:
            self._watchdog = threading.Thread(target=self._watch, args=(watchdog_s,), daemon=True)
            self._watchdog.start()
        if control is not None:
            control.attach(self)

    # ------------------------------------------------------------- roles --
    def coordinator_rank(self) -> int:
        return max(self.eg.members)

    def is_coordinator(self) -> bool:
        return self.eg.grank == self.coordinator_rank()

    # ------------------------------------------------------------ inputs --
    def submit_local(self, model: str, n_images: int = 0, images: Optional[List[str]] = None,
                     requester: str = "local", reply: Optional[Callable[[dict], None]] = None) -> None:
        """Queue a submit on the coordinator (applied at the next step)."""
        names = list(images) if images is not None else synthetic_names(n_images)
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

    # ----------------------------------------------------------- results --
    def _completed_local(self):
        """The oldest launched batch if its GPU work has finished (non-blocking)."""
        if not self.local:
            return None
        key, res, ev = self.local[0]
        if ev is not None and not ev.query():
            return None
        return self.local.popleft()

    def _exchange(self) -> List[Tuple[tuple, np.ndarray]]:
        """All-gather at most one completed batch per rank -> [(key, rows)]."""
        done = self._completed_local()
        sb = self.sbuf
        world, cap = self.eg.world, self.cap
        if self.comm is not None:
            ctx = torch.cuda.stream(self.comm)
        else:
            import contextlib

            ctx = contextlib.nullcontext()
        with ctx:
            sb[0, cap, :2] = -1
            if done is not None:
                key, res, ev = done
                if ev is not None and self.comm is not None:
                    self.comm.wait_event(ev)  # (already fired: ordering for the comm stream only)
                sb[:, :cap].copy_(res.to(self.dev))
                sb[0, cap, 0], sb[0, cap, 1] = int(key[0]), int(key[1])
            out = torch.empty((world, *sb.shape), dtype=sb.dtype, device=self.dev)
            self.eg.all_gather_into(out, sb)
            host = out.cpu().numpy()
        got = []
        for r in range(world):
            j, b = int(host[r, 0, cap, 0]), int(host[r, 0, cap, 1])
            if j >= 0:
                got.append(((j, b), host[r, :, :cap]))
        return got

    def _output_written(self, b: Batch) -> None:
        """(writer thread) A job is reported finished to its requester only once
        every batch's output file is durable — like the reference worker, which
        PUT its output before ACKing (worker.py:518-537) — so get-output right
        after the SUCCESS sees all of them."""
        with self.coord.lock:
            got = self._written.setdefault(b.job_id, set())
            got.add(b.batch_id)
            j = self.coord.jobs.jobs.get(b.job_id)
            ready = j is not None and j.done and len(got) >= j.batches_total
        if ready and self.control is not None:
            self.control.jobs_progress([b])

    # -------------------------------------------------------------- step --
    def step(self, stop_when_idle: bool = False) -> bool:
        eg, coord = self.eg, self.coord
        k = self.steps
        world = eg.world
        root = eg.group_rank_of(self.coordinator_rank())
        ph, t0 = self.phase_s, time.perf_counter()
        hcpu = np.zeros(HDR + world * DESC_FIELDS, np.int64)
        active = self.is_coordinator()
        payload = b""
        recs: List[dict] = []
        applied_here: List[dict] = []
        replies: List[Optional[Callable]] = []
        results: List[dict] = []
        if active:
            recs, replies = self._drain()
            with coord.lock:
                results = [coord.apply(r) for r in recs]
                stop = self._stop or (stop_when_idle and coord.idle() and not recs)
                table = coord.next_table(eg.members) if not stop else None
            if recs:
                payload = json.dumps(recs).encode()
            hcpu[0] = len(payload)
            hcpu[1] = k
            hcpu[2] = 1 if stop else 0
            if table is not None:
                hcpu[HDR:] = table.reshape(-1)
        t1 = time.perf_counter()
        ph["plan"] += t1 - t0
        with (torch.cuda.stream(self.comm) if self.comm is not None else _null()):
            hdr = torch.from_numpy(hcpu).to(self.dev)  # staged on the comm stream itself
            eg.broadcast(hdr, src=root)
            h = hdr.cpu().numpy()
            n = int(h[0])
            if n:
                buf = torch.zeros(n, dtype=torch.uint8, device=self.dev)
                if active:
                    buf.copy_(torch.frombuffer(bytearray(payload), dtype=torch.uint8))
                eg.broadcast(buf, src=root)
                if not active:
                    applied_here = json.loads(bytes(buf.cpu().numpy()).decode())
                    with coord.lock:
                        for r in applied_here:
                            coord.apply(r)
        applied = recs if active else applied_here
        for r in applied:  # collective on every rank: decode-once + replicate the job's images
            if r["op"] == "submit" and hasattr(self.be, "on_submit"):
                self.be.on_submit(r["model"], r["images"], eg)
        if active and self.control is not None:
            self.control.committed(replies, results)
        elif active:
            for cb, r in zip(replies, results):
                if cb is not None:
                    cb(r)
        t2 = time.perf_counter()
        ph["broadcast"] += t2 - t1
        if int(h[2]) == 1:  # STOP (sent only when nothing is queued or in flight)
            return False
        table = h[HDR:].reshape(world, DESC_FIELDS)
        with coord.lock:
            coord.apply_table(table, eg.members)
            mine = coord.assigned(table, eg.members, eg.grank)
        if k == self.kill_at_step and eg.grank == self.kill_rank:
            log.warning("rank %d: injected kill at step %d", eg.grank, k)
            os._exit(17)
        if mine is not None:
            res, ev = self.be.launch(mine.model, mine.images, self.launched % 2)
            self.launched += 1
            self.local.append((mine.key, res, ev))
        t3 = time.perf_counter()
        ph["launch"] += t3 - t2
        got = self._exchange()
        t4 = time.perf_counter()
        ph["exchange"] += t4 - t3
        if got:
            with coord.lock:
                finished = [coord.complete(key, rows) for key, rows in got]
            if self.is_coordinator():
                done = [d for d in finished if d is not None]
                for b, idx, p, g in done:
                    if self.writer is not None:
                        self.writer.submit(b, idx, p, g, on_written=self._output_written)
                if self.control is not None and self.writer is None:
                    self.control.jobs_progress([d[0] for d in done])
        self.steps += 1
        self.last_progress = time.monotonic()
        t5 = time.perf_counter()
        ph["complete"] += t5 - t4
        if not got and mine is None and not n:
            # nothing moved: poll again soon while GPUs work, back off when idle
            time.sleep(self.poll_sleep if coord.inflight else self.idle_sleep)
            ph["sleep"] += time.perf_counter() - t5
        return True

    # -------------------------------------------------------------- serve --
    def serve(self, max_steps: int = 10 ** 9, stop_when_idle: bool = False) -> int:
        while self.steps < max_steps:
            try:
                if not self.step(stop_when_idle):
                    break
            except CollectiveFailure as e:
                self._recover(e)
        if self.writer is not None:
            self.writer.flush()
        return self.steps

    def _recover(self, e: Exception) -> None:
        eg = self.eg
        log.warning("rank %d: collective failed (%s); rebuilding", eg.grank, e)
        with self.coord.lock:
            self.coord.requeue_inflight()
        deadline = time.monotonic() + 10
        while not (eg.dead & set(eg.members)) and time.monotonic() < deadline:
            time.sleep(0.01)  # let SWIM confirm who died
        was = self.coordinator_rank()
        eg.rebuild(set(eg.dead))  # aborts the communicator first (RCCL: ncclCommAbort)
        # the requeued batches' GPU work may still be running: let it drain before
        # their slots are reused (compute streams only; the aborted comm stream is not waited on)
        for st in (getattr(self.be, "stream", None), getattr(self.be, "copy_stream", None)):
            if st is not None:
                st.synchronize()
        self.local.clear()
        self.rebuilds += 1
        # the new coordinator's state is authoritative: replicas that completed one
        # exchange more or less than it did are repaired by a state record
        if self.is_coordinator():
            with self.coord.lock:
                snap = self.coord.jobs.snapshot()
            with self._inbox.mutex:
                self._inbox.queue.appendleft(({"op": "state", "jobs": snap}, None))
            if was != eg.grank and self.writer is not None:  # takeover: re-PUT recent outputs
                for b, idx, p, g in list(self.coord.history.values()):
                    self.writer.submit(b, idx, p, g, on_written=self._output_written)
            if self.control is not None:
                self.control.became_coordinator(was)
        self.last_progress = time.monotonic()

    def _watch(self, limit_s: float) -> None:
        """Watchdog: a rank whose serve loop makes no progress for ``limit_s``
        (e.g. stuck inside a collective the abort could not release) exits
        non-zero; it is never re-exec'ed (the survivors rebuild without it)."""
        while True:
            time.sleep(min(1.0, limit_s / 4))
            if time.monotonic() - self.last_progress > limit_s:
                log.error("rank %d: no progress for %.0f s, exiting", self.eg.grank, limit_s)
                os._exit(3)


def _null():
    import contextlib

    return contextlib.nullcontext()


# ------------------------------------------------------------ control plane ----
class RankControl:
    """This rank's host control plane, in a daemon thread with its own asyncio
    loop: a cluster Node with role "rank" (SWIM membership -> dead ranks for the
    elastic group, bully election -> store leader = coordinator, the replicated
    store with its TCP blob plane) plus the job-service request handlers the
    reference leader served (SUBMIT_JOB_REQUEST, C1, C2, C3 = SET_BATCH_SIZE,
    C5 = GET_ASSIGNMENTS, JOB_STATUS; worker.py:887-1059). Requests reach the
    serve loop through its inbox; replies go out once the request's log record
    has been broadcast (committed on every rank)."""

    def __init__(self, grank: int, world: int, base_port: int, store_dir: str, host: str = "127.0.0.1",
                 period: float = 0.1, ping_timeout: float = 0.1, suspect_timeout: float = 0.6,
                 replication: int = 4, on_dead: Optional[Callable[[int], None]] = None):
        self.grank, self.world, self.base, self.host = grank, world, base_port, host
        self.store_dir, self.replication = store_dir, replication
        self.period, self.ping_timeout, self.suspect_timeout = period, ping_timeout, suspect_timeout
        self.on_dead = on_dead
        self.svc: Optional[CollectiveService] = None
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.node = None
        self.ready = threading.Event()
        self.dead: set = set()
        self.thread = threading.Thread(target=self._main, daemon=True, name=f"rank-control-{grank}")

    def addr(self, g: int) -> str:
        return f"{self.host}:{self.base + g}"

    def rank_of(self, name: str) -> Optional[int]:
        try:
            return int(name.rsplit(":", 1)[1]) - self.base
        except (ValueError, IndexError):
            return None

    # ------------------------------------------------------------ thread --
    def start(self, timeout: float = 30.0) -> "RankControl":
        self.thread.start()
        if not self.ready.wait(timeout):
            raise RuntimeError("rank control plane did not start")
        return self

    def _main(self) -> None:
        self.loop = asyncio.new_event_loop()
        asyncio.set_event_loop(self.loop)
        self.loop.create_task(self._run())
        self.loop.run_forever()
        pending = [t for t in asyncio.all_tasks(self.loop) if not t.done()]
        for t in pending:
            t.cancel()
        if pending:
            self.loop.run_until_complete(asyncio.gather(*pending, return_exceptions=True))
        self.loop.close()

    async def _run(self) -> None:
        from ..cluster.frames import MsgType
        from ..serving.node import Node, NodeConfig

        cfg = NodeConfig(host=self.host, port=self.base + self.grank, role="rank", seeds=[self.addr(0)],
                         store_dir=self.store_dir, period=self.period, ping_timeout=self.ping_timeout,
                         suspect_timeout=self.suspect_timeout, cleanup_time=30.0, replication=self.replication,
                         meta={"prio": self.grank, "rank": self.grank})
        self.node = n = await Node(cfg).start()
        on = n.ep.on
        on(MsgType.SUBMIT_JOB_REQUEST, self._on_submit)
        on(MsgType.SET_BATCH_SIZE, self._on_batch_size)
        on(MsgType.GET_C1_COMMAND, self._on_c1)
        on(MsgType.GET_C2_COMMAND, self._on_c2)
        on(MsgType.GET_ASSIGNMENTS, self._on_c5)
        on(MsgType.JOB_STATUS, self._on_status)
        on(MsgType.FETCH_INTRODUCER, self._on_fetch_leader)   # every rank is an introducer for clients
        n.ml.on_fail.append(self._member_failed)
        await n.join()
        # every rank knows the static job membership: once all have joined, the
        # bully election settles on the highest rank (= the collective
        # coordinator); serving starts only then, so store requests of the first
        # steps already reach the right leader
        want = self.addr(self.world - 1)
        for _ in range(400):
            if len([m for m in n.ml.alive() if (n.ml.get(m).meta or {}).get("role") == "rank"]) >= self.world:
                break
            await asyncio.sleep(0.05)
        for _ in range(400):
            if n.leader() == want:
                break
            if not n.election.in_election:
                n.election.trigger()
            await asyncio.sleep(0.05)
        self.ready.set()

    def _member_failed(self, name: str) -> None:
        g = self.rank_of(name)
        if g is not None and 0 <= g < self.world and g not in self.dead:
            self.dead.add(g)
            log.warning("rank %d: SWIM confirmed rank %d dead", self.grank, g)
            if self.on_dead is not None:
                self.on_dead(g)

    def stop(self) -> None:
        if self.loop is None or not self.thread.is_alive():
            return

        async def _shutdown():
            try:
                await self.node.stop()
            except Exception:
                pass
            tasks = [t for t in asyncio.all_tasks() if t is not asyncio.current_task()]
            for t in tasks:
                t.cancel()
            await asyncio.gather(*tasks, return_exceptions=True)
        try:
            asyncio.run_coroutine_threadsafe(_shutdown(), self.loop).result(timeout=5)
        except Exception:
            pass
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.thread.join(timeout=5)

    # ------------------------------------------------------- serve hooks --
    def attach(self, svc: CollectiveService) -> None:
        self.svc = svc

    def call(self, coro, timeout: float = 30.0):
        """Run a coroutine on the control loop from the serve thread."""
        return asyncio.run_coroutine_threadsafe(coro, self.loop).result(timeout)

    def committed(self, replies: List[Optional[Callable]], results: List[dict]) -> None:
        for cb, r in zip(replies, results):
            if cb is not None:
                self.loop.call_soon_threadsafe(cb, r)

    def jobs_progress(self, batches: List[Batch]) -> None:
        """Tell requesters whose job just finished (SUBMIT_JOB_REQUEST_SUCCESS)."""
        from ..cluster.frames import MsgType

        seen = set()
        for b in batches:
            j = self.svc.coord.jobs.jobs.get(b.job_id)
            if j is not None and j.done and j.job_id not in seen and ":" in j.requester:  # a node, not "local"
                seen.add(j.job_id)
                self.loop.call_soon_threadsafe(
                    lambda jj=j: self.loop.create_task(
                        self.node.ep.send(jj.requester, MsgType.SUBMIT_JOB_REQUEST_SUCCESS, {"jobid": jj.job_id})))

    def became_coordinator(self, previous: int) -> None:
        log.warning("rank %d: now the coordinator (was rank %d)", self.grank, previous)
        # requesters of jobs that finished while the old coordinator was dying are told again
        done = [j for j in self.svc.coord.jobs.jobs.values() if j.done]
        self.jobs_progress([Batch(j.job_id, 0, j.model, []) for j in done])

    def store_put(self, name: str, data: bytes, deadline_s: float = 60.0) -> None:
        """PUT into the store, retried across a store-leader change (the leader
        is the coordinator rank, which is what fails over)."""
        t0, err = time.monotonic(), ""
        while time.monotonic() - t0 < deadline_s:
            try:
                ok, err = self.call(self.node.store.put(data, name), timeout=30)
            except Exception as e:  # leader unreachable mid-failover
                ok, err = False, str(e)
            if ok:
                return
            time.sleep(0.1)
        raise RuntimeError(f"store put {name}: {err}")

    def store_loader(self, names: List[str]) -> Dict[str, Optional[bytes]]:
        async def fetch_all():
            sem = asyncio.Semaphore(16)

            async def one(nm):
                async with sem:
                    if self.node.local.has(nm):
                        return nm, self.node.local.get_bytes(nm)
                    got = await self.node.store.get(nm)
                    return nm, None if got is None else got[1]
            return dict(await asyncio.gather(*(one(nm) for nm in names)))
        return self.call(fetch_all(), timeout=120)

    # ----------------------------------------------------------- handlers --
    async def _on_fetch_leader(self, fr) -> None:
        """Reference FETCH_INTRODUCER (introduce process/worker.py:55-58): any rank
        tells a client who leads, once the election has settled."""
        from ..cluster.frames import MsgType

        if self.ready.is_set() and self.node.leader() is not None:
            await self.node.ep.reply(fr, MsgType.FETCH_INTRODUCER_ACK, {"introducer": self.node.leader()})

    def _active(self) -> bool:
        return self.svc is not None and self.svc.is_coordinator()

    async def _on_submit(self, fr) -> None:
        from ..cluster.frames import MsgType

        if not self._active():
            return  # not the coordinator: the client retries at the elected leader
        p = fr.payload
        model = p["model"]
        n = int(p["images_count"])
        if p.get("synthetic"):
            names = synthetic_names(n)
        else:
            from ..serving.jobs import pick_images

            names = pick_images(sorted(self.node.store.meta.matching("*.jpeg")), n)

        def reply(res, fr=fr):
            self.loop.create_task(self.node.ep.reply(fr, MsgType.SUBMIT_JOB_REQUEST_ACK, res))
            if res.get("batches") == 0:
                self.loop.create_task(self.node.ep.send(fr.sender, MsgType.SUBMIT_JOB_REQUEST_SUCCESS,
                                                        {"jobid": res["jobid"]}))
        self.svc.submit_local(model, images=names, requester=fr.sender, reply=reply)

    async def _on_batch_size(self, fr) -> None:
        from ..cluster.frames import MsgType

        if not self._active():
            return

        def reply(res, fr=fr):
            if fr.seq:
                self.loop.create_task(self.node.ep.reply(fr, MsgType.SET_BATCH_SIZE_ACK, res))
        self.svc.set_batch_size(fr.payload["model"], int(fr.payload["batch_size"]), reply=reply)

    async def _on_c1(self, fr) -> None:
        from ..cluster.frames import MsgType

        if self._active():
            with self.svc.coord.lock:
                c1 = self.svc.coord.metrics.c1()
            await self.node.ep.reply(fr, MsgType.GET_C1_COMMAND_ACK, {"c1": c1})

    async def _on_c2(self, fr) -> None:
        from ..cluster.frames import MsgType

        if self._active():
            with self.svc.coord.lock:
                p = self.svc.coord.metrics.c2_reference_payload()
                p["detail"] = self.svc.coord.metrics.c2()
            await self.node.ep.reply(fr, MsgType.GET_C2_COMMAND_ACK, p)

    async def _on_c5(self, fr) -> None:
        from ..cluster.frames import MsgType

        if self._active():
            with self.svc.coord.lock:
                a = self.svc.coord.assignments()
            await self.node.ep.reply(fr, MsgType.GET_ASSIGNMENTS_ACK, {"assignments": a})

    async def _on_status(self, fr) -> None:
        from ..cluster.frames import MsgType

        if not self._active():
            return
        with self.svc.coord.lock:
            j = self.svc.coord.jobs.jobs.get(int(fr.payload["jobid"]))
            st = {"jobid": fr.payload["jobid"], "known": j is not None, "done": bool(j and j.done),
                  "batches_done": j.batches_done if j else 0, "batches_total": j.batches_total if j else 0}
        await self.node.ep.reply(fr, MsgType.JOB_STATUS_ACK, st)
