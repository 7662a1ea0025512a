"""HBM-resident decoded-image store, staged in sliding windows ahead of dispatch and
replicated across the ranks over the data group (RCCL on a GPU node).

Reference: SDFS keeps every JPEG on 4 replicas (``leader.py:45-85``), copied by
scp (``file_service.py:52-124``), and every worker scp-downloads and decodes each
image of its batch again, one at a time, when the task arrives
(``worker.py:1361-1386``) — any job size works because nothing is held beyond a batch.

MI355X-native replacement (SURVEY §2.6 "replication multicast" row):

* a job's images are staged in WINDOWS that run just ahead of dispatch: every
  step the service hands the batches about to be dispatched (and any dispatched
  batch not staged yet) to ``stage``; their not-yet-resident images form one
  window. Every rank takes the same decisions from the replicated job state
  (same queue order, same arena bookkeeping), so windows, slot assignments and
  evictions are identical everywhere without any extra agreement;
* a window's images are fetched (store blob plane) and DECODED ONCE IN THE WHOLE
  JOB — image i of the window by rank i % world, in a host thread pool, off the
  serve loop — then replicated to every rank's HBM with one all-gather over the
  data group, issued asynchronously from the serve loop (windows in the same
  order on every rank) and followed, in stream order, by the scatter into the
  window's arena slots and an event: a batch launches once its window's event is
  recorded (the compute stream waits on it), so the serve loop never blocks on
  staging;
* arena slots are pinned by the staged, unfinished batches that use them
  (refcounts) and released when a batch completes; eviction takes the oldest
  unpinned image; a window that does not fit waits for completions. Any job size
  runs in a fixed arena (``capacity`` >= the images of the batches in flight);
* an image that could not be fetched or decoded is failed for the batches of its
  window only: it is forgotten when its last batch completes, and a later job
  fetches it again (a transient store miss during a leader fail-over is not
  permanent);
* after any epoch change (failure rebuild, rejoin) every rank drops its staging
  state at the same step boundary (``reset``) and the windows are staged afresh
  for the new member set — a re-joined rank needs no special backfill.
"""
from __future__ import annotations

import logging
from collections import OrderedDict, deque
from dataclasses import dataclass, field
from typing import Callable, Deque, Dict, List, Optional, Sequence, Set, Tuple

import numpy as np
import torch

log = logging.getLogger(__name__)
SYNTH = "synthetic:"


@dataclass
class Window:
    store: "HbmImageStore"
    wid: int
    epoch: int
    names: List[str]          # the new images of this window (replicated by it)
    slots: List[int]          # their arena slots (decided by plan, identical on every rank)
    mine: List[str] = field(default_factory=list)      # this rank's decode share
    future: Optional[object] = None                    # decode of this rank's share (thread pool)
    work: Optional[list] = None                        # pending async collectives (gloo: polled)
    bufs: Optional[tuple] = None                       # (send, recv, ok_send, ok_recv) tensors
    event: Optional[object] = None                     # recorded after the scatter (CUDA)
    flags: Optional[torch.Tensor] = None               # ok flag per gathered row (host)
    src: Optional[List[int]] = None                    # gathered row of each name
    failed: Set[str] = field(default_factory=set)
    done: bool = False


class HbmImageStore:
    """One model's arena of decoded uint8 images [capacity, H, W, 3] (HBM on a GPU
    rank; host memory in CPU tests) + the window bookkeeping described above."""

    def __init__(self, capacity: int, hw: Tuple[int, int], device: torch.device, n_synth: int = 0,
                 seed: int = 0):
        if n_synth >= capacity:
            raise ValueError("arena needs room beyond its synthetic images")
        self.capacity, self.hw, self.device, self.n_synth = capacity, tuple(hw), torch.device(device), n_synth
        self.arena = torch.zeros((capacity, *self.hw, 3), dtype=torch.uint8, device=self.device)
        if n_synth:  # seeded, identical on every rank
            rng = np.random.default_rng(seed)
            for i in range(0, n_synth, 64):
                j = min(n_synth, i + 64)
                self.arena[i:j].copy_(torch.from_numpy(rng.integers(0, 256, size=(j - i, *self.hw, 3),
                                                                    dtype=np.uint8)))
        self.loader: Optional[Callable] = None   # names -> {name: uint8 HxWx3 | None} (decode pool)
        self.stager = Stager()  # replaced by the backend's shared one (one collective order for all models)
        self.reset()
        self.decoded = 0        # images this rank decoded
        self.replicated = 0     # images that arrived in this rank's arena
        self.windows_staged = 0
        self.evictions = 0

    # ----------------------------------------------------------- state --
    def reset(self) -> None:
        """Forget every staged image (epoch change): identical on every rank."""
        self.index: "OrderedDict[str, int]" = OrderedDict()   # name -> slot, in staging (FIFO) order
        self.window_of: Dict[str, Window] = {}                 # name -> the window that stages it
        self.refs: Dict[str, int] = {}
        self.free: List[int] = list(range(self.capacity - 1, self.n_synth - 1, -1))
        self._wid = 0

    def _synthetic(self, n: str) -> bool:
        return self.n_synth > 0 and n.startswith(SYNTH)

    def resident(self, name: str) -> bool:
        return name in self.index

    # ------------------------------------------------- plan (deterministic) --
    def plan(self, names: Sequence[str], epoch: int) -> Optional[Window]:
        """(serve loop, every rank, same order) reserve slots for the images of
        ``names`` that are not staged yet; None if they do not fit next to the
        pinned images (the caller stages fewer batches and retries later). Returns
        the window (possibly with no new names)."""
        new = [n for n in dict.fromkeys(names) if not self._synthetic(n) and n not in self.index]
        if len(new) > len(self.free) + sum(1 for k in self.index if self.refs.get(k, 0) == 0 and k not in new):
            return None
        slots = []
        for n in new:
            if not self.free:  # evict the oldest unpinned image
                victim = next(k for k in self.index if self.refs.get(k, 0) == 0)
                self.free.append(self.index.pop(victim))
                self.window_of.pop(victim, None)
                self.evictions += 1
            s = self.free.pop()
            slots.append(s)
            self.index[n] = s
        w = Window(self, self._wid, epoch, new, slots)
        self._wid += 1
        for n in new:
            self.window_of[n] = w
        if new:
            self.stager.queue.append(w)
            self.windows_staged += 1
        else:
            w.done = True
        return w

    def pin(self, names: Sequence[str]) -> None:
        for n in names:
            if not self._synthetic(n):
                self.refs[n] = self.refs.get(n, 0) + 1

    def unpin(self, names: Sequence[str]) -> None:
        """A batch completed (same step on every rank). Its images stay resident
        (evictable once unpinned) — except failed ones, which are forgotten so a
        later window fetches them again."""
        for n in names:
            if self._synthetic(n):
                continue
            r = self.refs.get(n, 0) - 1
            if r > 0:
                self.refs[n] = r
                continue
            self.refs.pop(n, None)
            w = self.window_of.get(n)
            if w is None:
                continue
            if not w.done:
                # every rank decides this at the same step: a batch of w completed somewhere,
                # so every rank has issued w's collective and finishing it here is bounded
                self.stager.flush_until(w)
            if n in w.failed and n in self.index:
                self.free.append(self.index.pop(n))
                self.window_of.pop(n, None)

    # --------------------------------------------------------- readiness --
    def ready(self, names: Sequence[str]) -> bool:
        for n in names:
            if self._synthetic(n):
                continue
            w = self.window_of.get(n)
            if w is None or not w.done:
                return False
        return True

    def events(self, names: Sequence[str]) -> List[object]:
        evs = {id(w.event): w.event for w in (self.window_of.get(n) for n in names)
               if w is not None and w.event is not None}
        return list(evs.values())

    def slots(self, names: Sequence[str]) -> Tuple[List[int], List[str]]:
        """Arena slots of a staged batch; failed images get slot 0 and are listed."""
        out, failed = [], []
        for n in names:
            if self._synthetic(n):
                out.append(int(n[len(SYNTH):]) % self.n_synth)
                continue
            w = self.window_of.get(n)
            if n not in self.index or w is None or n in w.failed:
                failed.append(n)
                out.append(0)
            else:
                out.append(self.index[n])
        return out, failed

    # ------------------------------------------------------ replication --
    def _issue(self, w: Window, rank: int, world: int, got: Dict[str, Optional[np.ndarray]],
               gather_async: Callable, stream) -> None:
        chunk = max(1, -(-len(w.names) // world))
        stage = torch.zeros((chunk, *self.hw, 3), dtype=torch.uint8)
        ok = torch.zeros(chunk, dtype=torch.int32)
        for j, n in enumerate(w.mine):
            img = got.get(n)
            if img is not None:
                stage[j].numpy()[...] = img  # loader arrays may be read-only views
                ok[j] = 1
        self.decoded += int(ok.sum())
        ctx = torch.cuda.stream(stream) if (stream is not None and self.device.type == "cuda") else _null()
        with ctx:
            if self.device.type == "cuda":
                send = stage.pin_memory().to(self.device, non_blocking=True)
                okd = ok.pin_memory().to(self.device, non_blocking=True)
            else:
                send, okd = stage, ok
            if world == 1:
                w.bufs, w.work = (send, send, okd, okd), []
                return
            recv = torch.empty((world * chunk, *self.hw, 3), dtype=torch.uint8, device=self.device)
            okr = torch.empty(world * chunk, dtype=torch.int32, device=self.device)
            w.bufs = (send, recv, okd, okr)
            w.work = [gather_async(recv, send), gather_async(okr, okd)]

    def _finish(self, w: Window, world: int, stream) -> bool:
        """Once the window's collective is in place: scatter every name's row into its
        slot (stream order on a GPU; failed rows are zeros) and bring the ok flags to the
        host asynchronously; the window is done (ready to launch from) when they arrive."""
        cuda = self.device.type == "cuda"
        if w.event is None:
            if not cuda and any(not wk.is_completed() for wk in w.work):
                return False
            send, recv, okd, okr = w.bufs
            chunk = okr.numel() // world
            ctx = torch.cuda.stream(stream) if (stream is not None and cuda) else _null()
            with ctx:
                for wk in w.work:
                    try:
                        wk.wait()  # gloo: completed already; RCCL: the staging stream waits on it
                    except Exception as e:  # a peer died mid-collective: the serve loop recovers
                        from .elastic import CollectiveFailure

                        raise CollectiveFailure(f"image window collective failed: {e}") from e
                src = [(i % world) * chunk + i // world for i in range(len(w.names))]
                self.arena.index_copy_(0, torch.tensor(w.slots, device=self.device),
                                       recv.index_select(0, torch.tensor(src, device=self.device)))
                if cuda:
                    w.flags = okr.to("cpu", non_blocking=True) if okr.is_cuda else okr
                    w.event = torch.cuda.Event()
                    w.event.record()
                else:
                    w.flags, w.event = okr, True
            w.src = src
        if cuda and not w.event.query():
            return False
        flags = w.flags.numpy()
        for n, k in zip(w.names, w.src):
            if not flags[k]:
                w.failed.add(n)
        self.replicated += len(w.names) - len(w.failed)
        if not cuda:
            w.event = None
        w.bufs, w.work, w.flags, w.done = None, None, None, True
        return True


class Stager:
    """The windows of every model's store in ONE plan order: their all-gathers go out
    on the data group in that order on every rank (gloo / RCCL match collectives by
    order, so two models' windows must never be issued in a rank-dependent order)."""

    def __init__(self):
        self.queue: Deque[Window] = deque()
        self.ctx = (0, 1, None, None, None)
        self.poll_dead: Callable[[], None] = lambda: None

    def attach(self, rank: int, world: int, pool, gather_async: Callable, stream=None,
               poll_dead: Optional[Callable[[], None]] = None) -> None:
        """The group the windows replicate over (every epoch): group rank / size, the decode
        pool, the async all-gather, the staging stream; ``poll_dead`` raises CollectiveFailure
        once a member is confirmed dead (a blocking flush polls it: a collective with a dead
        peer never completes on RCCL, and a hung peer keeps gloo's sockets open)."""
        self.ctx = (rank, world, pool, gather_async, stream)
        self.poll_dead = poll_dead or (lambda: None)

    def flush_until(self, target: Window) -> None:
        """Block until ``target`` (and every window before it) is resident here."""
        import time

        while not target.done and self.queue:
            w = self.queue[0]
            if w.future is not None and not w.future.done():
                w.future.result()
            # the window's collective / scatter: polled, never a blocking wait (a dead peer)
            while ((w.work is not None and w.event is None and w.store.device.type != "cuda"
                    and not all(wk.is_completed() for wk in w.work)) or
                   (w.event is not None and not isinstance(w.event, bool) and not w.event.query())):
                self.poll_dead()
                time.sleep(0.0002)
            if not self.progress():
                self.poll_dead()
                time.sleep(0.0005)

    def progress(self) -> int:
        """(serve loop, never blocks) advance the queued windows in order: start this
        rank's decode share, issue a window's all-gather once its decode finished (in plan
        order on every rank), finish windows whose collective completed. Returns the
        windows finished now."""
        rank, world, pool, gather_async, stream = self.ctx
        finished = 0
        for w in self.queue:  # decodes of every queued window may run ahead in the pool
            if w.future is None:
                w.mine = w.names[rank::world]
                w.future = pool.submit(_safe_load, w.store.loader, list(w.mine))
        while self.queue:
            w = self.queue[0]
            if w.work is None:
                if not w.future.done():
                    break
                w.store._issue(w, rank, world, w.future.result(), gather_async, stream)
            if not w.store._finish(w, world, stream):
                break
            self.queue.popleft()
            finished += 1
        return finished

    def drain(self) -> None:
        """Drop every queued window (epoch change; its collectives were aborted)."""
        for w in self.queue:
            if w.future is not None:
                w.future.cancel()
        self.queue.clear()


def _safe_load(load: Callable, names: List[str]) -> Dict[str, Optional[np.ndarray]]:
    """A loader exception (store unreachable mid fail-over, timeout) fails this share of
    the window's images, never the serve loop."""
    if not names:
        return {}
    try:
        return load(names)
    except Exception as e:
        log.warning("image fetch/decode of %d images failed: %s", len(names), e)
        return {n: None for n in names}


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
