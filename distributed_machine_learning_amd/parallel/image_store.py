"""HBM-resident decoded-image store, staged in windows ahead of dispatch and delivered only
to the rank that runs each batch (RCCL over the data group on a GPU node).

Reference: SDFS keeps every JPEG on 4 replicas (``leader.py:45-85``), copied by
scp (``file_service.py:52-124``), and every worker scp-downloads and decodes each
image of its batch again, one at a time, when the task arrives
(``worker.py:1361-1386``) — any job size works because nothing is held beyond a batch.

MI355X-native replacement (SURVEY §2.6 "replication multicast" row):

* a batch's images are staged in a WINDOW for ONE destination rank — the rank the batch
  is dispatched to, or, for a batch still queued, the rank the replicated coordinator
  gave it as its affinity (``ReplicatedCoordinator.assign_affinity``; the plan then
  dispatches the batch there). Every rank takes the same decisions from the replicated
  job state (same queue order, same arena bookkeeping, same slot map), so windows, slot
  assignments and evictions are identical everywhere without any extra agreement; only
  the pixels differ: a slot holds its image on the ranks that hold it (``holders``);
* an image new to the job is fetched (store blob plane) and DECODED ONCE, by the
  destination rank itself, in a host thread pool off the serve loop — nothing crosses
  xGMI for it. An image another rank already holds (a cyclic job re-using its images, a
  batch re-dispatched away from its affinity rank) is SHIPPED from the lowest holder's
  arena by an uneven all-to-all over the data group — HBM to HBM, no second decode —
  never all-gathered to every rank (all-gather-to-all moved world x
  the needed bytes). Each window also all-reduces one ok flag per image (a few bytes),
  so every rank learns the failures and keeps identical bookkeeping;
* the collectives are issued asynchronously from the serve loop, in plan order on every
  rank, and followed, in stream order, by the scatter into the window's arena slots and
  an event: a batch launches once the windows that delivered its images HERE are done
  (the compute stream waits on their events), so the serve loop never blocks on staging;
* arena slots are pinned by the staged, unfinished batches that use them (refcounts) and
  released when a batch completes; eviction takes the oldest unpinned image; a window
  that does not fit waits for completions. Any job size runs in a fixed arena;
* an image that could not be fetched or decoded is failed for the batches of its window
  only: it is forgotten when its last batch completes, and a later job fetches it again
  (a transient store miss during a leader fail-over is not permanent);
* after any epoch change (failure rebuild, rejoin) every rank drops its staging state at
  the same step boundary (``reset``) and the windows are staged afresh for the new member
  set — a re-joined rank needs no special backfill. (A spare copy on a second rank would
  therefore buy nothing on failover: the survivors re-stage from the store either way.)
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
    dst: int                  # the group rank these images become resident on
    names: List[str]          # images this window makes resident on dst (new + shipped)
    slots: List[int]          # their arena slots (decided by plan, identical on every rank)
    src: List[int]            # per name: the rank that supplies it (== dst: decoded there)
    mine: List[str] = field(default_factory=list)      # this rank's decode share (dst == this rank)
    future: Optional[object] = None                    # decode of this rank's share (thread pool)
    work: Optional[list] = None                        # pending async collectives (gloo: polled)
    bufs: Optional[tuple] = None                       # (local rows, received rows, flags) tensors
    event: Optional[object] = None                     # recorded after the scatter (CUDA)
    flags: Optional[torch.Tensor] = None               # ok flag per name (host), after the all-reduce
    pack: Optional[object] = None                      # GPU backend: the pinned pack of its decodes
    failed: Set[str] = field(default_factory=set)
    done: bool = False
    deps: List["Window"] = field(default_factory=list)  # earlier unfinished windows writing one of its slots
    # rows this rank ships (it is their lowest holder): row index -> the window that delivered the
    # image HERE. The row's ok flag is that window's final flag, so the ship window is not issued
    # before it is done (an issue-ahead ship read an empty ``failed`` set)
    ship_src: Dict[int, "Window"] = field(default_factory=dict)

    @property
    def shipped(self) -> int:
        return sum(1 for s in self.src if s != self.dst)


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
        self.replicated = 0     # images that became resident in this rank's arena (decoded or shipped here)
        self.received = 0       # of those, shipped here from another rank's arena
        self.shipped_out = 0    # rows this rank's arena sent to other ranks
        self.windows_staged = 0
        self.evictions = 0

    @property
    def me(self) -> int:
        return self.stager.ctx[0]

    # ----------------------------------------------------------- state --
    def reset(self) -> None:
        """Forget every staged image (epoch change): identical on every rank."""
        self.index: "OrderedDict[str, int]" = OrderedDict()   # name -> slot, in staging (FIFO) order
        self.holders: Dict[str, Set[int]] = {}                 # name -> ranks it is (being) delivered to
        self.window_of: Dict[str, Window] = {}                 # name -> the latest window that moves it
        self.here: Dict[str, Window] = {}                      # name -> the window that delivers it HERE
        self.refs: Dict[str, int] = {}
        # resident images no batch pins (refs 0), least recently released first: the eviction
        # candidates, kept incrementally (plan() used to scan the whole index per batch with a
        # list membership test per entry: 258 ms steps at 51,200 distinct images)
        self.idle: "OrderedDict[str, None]" = OrderedDict()
        self.free: List[int] = list(range(self.capacity - 1, self.n_synth - 1, -1))
        self.slot_win: Dict[int, Window] = {}   # slot -> the latest window writing it
        self._wid = 0

    def _synthetic(self, n: str) -> bool:
        return self.n_synth > 0 and n.startswith(SYNTH)

    def resident(self, name: str, rank: Optional[int] = None) -> bool:
        """Staged (anywhere), or - with ``rank`` - staged for that rank."""
        if rank is None:
            return name in self.index
        return rank in self.holders.get(name, ())

    # ------------------------------------------------- plan (deterministic) --
    def plan(self, names: Sequence[str], epoch: int, dst: int = 0) -> Optional[Window]:
        """(serve loop, every rank, same order) make the images of ``names`` resident on
        group rank ``dst``: slots for the ones not staged anywhere (decoded by ``dst``), a
        shipment from a holder for the ones staged elsewhere; None if the new ones do not
        fit next to the pinned images (the caller stages fewer batches and retries later).
        Returns the window (possibly with no names)."""
        want = [n for n in dict.fromkeys(names) if not n.startswith(SYNTH)] if self.n_synth else list(dict.fromkeys(names))
        wset = set(want)
        new = [n for n in want if n not in self.index]
        move = [n for n in want if n in self.index and dst not in self.holders[n]]
        if len(new) > len(self.free) + len(self.idle) - sum(1 for n in want if n in self.idle):
            return None
        slots, src = [], []
        for n in new:
            if not self.free:  # evict the least recently released unpinned image
                victim = next(k for k in self.idle if k not in wset)
                del self.idle[victim]
                self.free.append(self.index.pop(victim))
                self.holders.pop(victim, None)
                self.window_of.pop(victim, None)
                self.here.pop(victim, None)
                self.evictions += 1
            s = self.free.pop()
            slots.append(s)
            src.append(dst)
            self.index[n] = s
            self.idle[n] = None   # unpinned until its batch pins it
            self.holders[n] = {dst}
        ship_src: Dict[int, Window] = {}
        for n in move:
            h = min(self.holders[n])           # the lowest holder ships it (its copy lands first)
            if h == self.me and n in self.here:
                ship_src[len(slots)] = self.here[n]
            slots.append(self.index[n])
            src.append(h)
            self.holders[n].add(dst)
        w = Window(self, self._wid, epoch, dst, new + move, slots, src, ship_src=ship_src)
        self._wid += 1
        deps = {}
        for s in slots:
            prev = self.slot_win.get(s)
            if prev is not None and not prev.done:
                deps[id(prev)] = prev
            self.slot_win[s] = w
        w.deps = list(deps.values())
        for n in w.names:
            self.window_of[n] = w
            if dst == self.me:
                self.here[n] = w
        if w.names:
            self.stager.queue.append(w)
            self.windows_staged += 1
        else:
            w.done = True
        return w

    def _real(self, names: Sequence[str]) -> Sequence[str]:
        """The store images of a batch (its synthetic rows live in the arena's seeded slots);
        one pass, not a method call per name (these run per batch on the serve loop)."""
        return [n for n in names if not n.startswith(SYNTH)] if self.n_synth else names

    def pin(self, names: Sequence[str]) -> None:
        refs, idle = self.refs, self.idle
        for n in self._real(names):
            r = refs.get(n, 0)
            if r == 0:
                idle.pop(n, None)
            refs[n] = r + 1

    def unpin(self, names: Sequence[str]) -> None:
        """A batch completed (same step on every rank). Its images stay resident
        (evictable once unpinned) — except failed ones, which are forgotten so a
        later window fetches them again."""
        for n in self._real(names):
            r = self.refs.get(n, 0) - 1
            if r > 0:
                self.refs[n] = r
                continue
            self.refs.pop(n, None)
            if n in self.index:
                self.idle[n] = None
            w = self.window_of.get(n)
            if w is None:
                continue
            if not w.done:
                # every rank decides this at the same step: a batch of w completed somewhere,
                # so every rank has issued w's collectives and finishing it here is bounded
                self.stager.flush_until(w)
            if n in w.failed and n in self.index:
                self.idle.pop(n, None)
                self.free.append(self.index.pop(n))
                self.holders.pop(n, None)
                self.window_of.pop(n, None)
                self.here.pop(n, None)

    # --------------------------------------------------------- readiness --
    def ready(self, names: Sequence[str]) -> bool:
        """Every image of a batch is resident on THIS rank."""
        here = self.here
        for n in self._real(names):
            w = here.get(n)
            if w is None or not w.done:
                return False
        return True

    def events(self, names: Sequence[str]) -> List[object]:
        evs = {id(w.event): w.event for w in (self.here.get(n) for n in names)
               if w is not None and w.event is not None}
        return list(evs.values())

    def slots(self, names: Sequence[str]) -> Tuple[List[int], List[str]]:
        """Arena slots of a batch staged here; failed images get slot 0 and are listed."""
        out, failed = [], []
        syn, here, index = self.n_synth > 0, self.here, self.index
        for n in names:
            if syn and n.startswith(SYNTH):
                out.append(int(n[len(SYNTH):]) % self.n_synth)
                continue
            w = here.get(n)
            if n not in index or w is None or n in w.failed:
                failed.append(n)
                out.append(0)
            else:
                out.append(self.index[n])
        return out, failed

    # ---------------------------------------------------------- delivery --
    def _issue(self, w: Window, rank: int, world: int, got: Dict[str, Optional[np.ndarray]], comm, stream) -> None:
        """This rank's part of window ``w``: its decoded images (dst), the rows it ships
        from its arena (a holder), the all-to-all of the shipped rows and the all-reduce of
        the ok flags (both skipped when nothing needs them: identical decisions everywhere)."""
        cuda = self.device.type == "cuda"
        okn = np.zeros(len(w.names), np.int32)   # numpy: a torch __setitem__ per image cost ~1 ms per window
        local = None
        pack = getattr(got, "pack", None)   # GPU backend: full-resolution decodes, resized on the GPU
        if rank == w.dst and w.mine and pack is None:
            local = torch.zeros((len(w.mine), *self.hw, 3), dtype=torch.uint8)
            for j, n in enumerate(w.mine):
                img = got.get(n)
                if img is not None:
                    local[j].numpy()[...] = img  # loader arrays may be read-only views
        if w.mine:
            good = [got.get(n) is not None for n in w.mine]
            if rank == w.dst:
                self.decoded += sum(good)
            if len(w.mine) == len(w.names) and w.mine == w.names:   # a window of new images only
                okn[:] = good
            else:
                pos = {n: i for i, n in enumerate(w.names)}
                okn[[pos[n] for n, g in zip(w.mine, good) if g]] = 1
        out_rows = [i for i, s in enumerate(w.src) if s == rank and s != w.dst]   # shipped from here
        for i in out_rows:
            mine = w.ship_src.get(i)   # done (Stager.progress holds the issue until it is)
            okn[i] = int(mine is not None and mine.done and w.names[i] not in mine.failed)
        ok = torch.from_numpy(okn)
        ctx = torch.cuda.stream(stream) if (stream is not None and cuda) else _null()
        with ctx:
            if cuda and local is not None:
                local = local.pin_memory().to(self.device, non_blocking=True)
            if pack is not None and rank == w.dst:
                # the decoded images land in their slots straight from the pinned pack (one H2D
                # copy + one resize kernel on the staging stream); no local rows to scatter
                slot_of = dict(zip(w.names, w.slots))
                # a pack may decode on a side stream of its own: it must not overtake an earlier
                # window still writing one of these slots (an evicted, never-pinned image)
                pack.after = self._slot_writer_events(w) if cuda else []
                pack.launch([slot_of[n] for n in pack.names], self.arena, stream)
                w.pack = pack
            recv, work = None, []
            if world > 1 and w.shipped:
                in_splits = [len(out_rows) if r == w.dst else 0 for r in range(world)]
                out_splits = [sum(1 for s in w.src if s == r and s != w.dst) if rank == w.dst else 0
                              for r in range(world)]
                send = (self.arena.index_select(0, torch.tensor([w.slots[i] for i in out_rows], device=self.device))
                        if out_rows else torch.empty((0, *self.hw, 3), dtype=torch.uint8, device=self.device))
                recv = torch.empty((sum(out_splits), *self.hw, 3), dtype=torch.uint8, device=self.device)
                work.append(comm.all_to_all_data_async(recv, send, out_splits, in_splits))
                self.shipped_out += len(out_rows)
            okd = ok.pin_memory().to(self.device, non_blocking=True) if cuda else ok
            if world > 1:
                work.append(comm.all_reduce_data_async(okd))
            w.bufs, w.work = (local, recv, okd), work

    def _slot_writer_events(self, w: Window) -> List[object]:
        """Events a window's GPU decode must wait on: per earlier unfinished window touching one
        of its slots, the decode's own completion event when that window only DECODED into the
        slot here (its side stream), else its staging-stream event (it scattered shipped rows
        into the slot, or read the slot to ship it). The staging-stream event has waited on every
        earlier window's decode, so using it for a decode-only writer chained the decodes again
        once the arena recycled slots."""
        evs: Dict[int, object] = {}
        mine = set(w.slots)
        for d in w.deps:
            if d.done:
                continue
            dec: Dict[str, object] = {}   # image -> the side-stream event of the decode that wrote it
            subs = getattr(d.pack, "packs", None) or ([d.pack] if d.pack is not None else [])
            for p in subs:
                if getattr(p, "done", None) is not None:
                    for n in p.names:
                        dec[n] = p.done
            for n, sl, sr in zip(d.names, d.slots, d.src):
                if sl not in mine:
                    continue
                ev = dec.get(n) if (d.dst == self.me and sr == d.dst) else None
                ev = ev if ev is not None else d.event
                if ev is not None:
                    evs[id(ev)] = ev
        return list(evs.values())

    def _finish(self, w: Window, world: int, stream) -> bool:
        """Once the window's collectives are in place: on its destination, scatter the
        decoded and the received rows into their slots (stream order on a GPU; failed rows
        are zeros); everywhere, bring the ok flags to the host asynchronously. The window is
        done (ready to launch from) when they arrive."""
        cuda = self.device.type == "cuda"
        if w.done:
            return True
        if w.event is None:
            if not cuda and any(not wk.is_completed() for wk in w.work):
                return False
            local, recv, okd = w.bufs
            ctx = torch.cuda.stream(stream) if (stream is not None and cuda) else _null()
            with ctx:
                for wk in w.work:
                    try:
                        wk.wait()  # gloo: completed already; RCCL: the staging stream waits on it
                    except Exception as e:  # a peer died mid-collective: the serve loop recovers
                        from .elastic import CollectiveFailure

                        raise CollectiveFailure(f"image window collective failed: {e}") from e
                if self.me == w.dst:
                    # received rows arrive grouped by source rank, each group in window order
                    order = [i for i, s in enumerate(w.src) if s == w.dst] if local is not None else []
                    order += [i for r in range(world) for i, s in enumerate(w.src) if s == r and s != w.dst]
                    rows = [t for t in (local, recv) if t is not None and t.shape[0]]
                    if rows:
                        data = rows[0] if len(rows) == 1 else torch.cat(rows)
                        self.arena.index_copy_(0, torch.tensor([w.slots[i] for i in order], device=self.device),
                                               data)
                if cuda:
                    w.flags = okd.to("cpu", non_blocking=True)
                    w.event = torch.cuda.Event()
                    w.event.record()
                else:
                    w.flags, w.event = okd, True
        if cuda and not w.event.query():
            return False
        flags = w.flags.numpy()
        for n, f in zip(w.names, flags):
            if not f:
                w.failed.add(n)
        if self.me == w.dst:
            arrived = len(w.names) - sum(1 for n in w.names if n in w.failed)
            self.replicated += arrived
            self.received += sum(1 for n, s in zip(w.names, w.src) if s != w.dst and n not in w.failed)
        if not cuda:
            w.event = None
        if w.pack is not None:   # its H2D copy and resize ran before the window's event
            w.pack.release()
            w.pack = None
        w.bufs, w.work, w.flags, w.done = None, None, None, True
        return True


class Stager:
    """The windows of every model's store in ONE plan order: their collectives go out on
    the data group in that order on every rank (gloo / RCCL match collectives by order, so
    two models' windows must never be issued in a rank-dependent order)."""

    def __init__(self):
        self.queue: Deque[Window] = deque()
        self.ctx = (0, 1, None, None, None)
        self.poll_dead: Callable[[], None] = lambda: None

    def attach(self, rank: int, world: int, pool, comm, stream=None,
               poll_dead: Optional[Callable[[], None]] = None) -> None:
        """The group the windows move over (every epoch): group rank / size, the decode
        pool, the data-group collectives (an ElasticGroup: all_to_all_data_async,
        all_reduce_data_async; None at world 1), the staging stream; ``poll_dead`` raises
        CollectiveFailure once a member is confirmed dead (a blocking flush polls it: a
        collective with a dead peer never completes on RCCL, and a hung peer keeps gloo's
        sockets open)."""
        self.ctx = (rank, world, pool, comm, stream)
        self.poll_dead = poll_dead or (lambda: None)

    def flush_until(self, target: Window) -> None:
        """Block until ``target`` (and every window before it) is done here."""
        import time

        while not target.done and self.queue:
            w = self.queue[0]
            if w.future is not None and not w.future.done():
                w.future.result()
            # the window's collectives / scatter: polled, never a blocking wait (a dead peer)
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
        rank's decodes (the windows it is the destination of), issue a window's
        collectives once its decode finished (in plan order on every rank), finish windows
        whose collectives completed. Returns the windows finished now."""
        rank, world, pool, comm, stream = self.ctx
        finished = 0
        for w in self.queue:  # decodes of every queued window may run ahead in the pool
            if w.future is None:
                w.mine = [n for n, s in zip(w.names, w.src) if s == w.dst] if rank == w.dst else []
                w.future = pool.submit(_safe_load, w.store.loader, list(w.mine))
        # issue every window whose decode finished, in plan order, without waiting for the
        # earlier windows to complete: issuing only after the previous window's event ran the GPU
        # JPEG decodes strictly one after the other (rocprofv3: 400 Huffman launches, 0 overlapped,
        # profiles/r5_store). On a GPU the scatter + event follow the issue at once (RCCL waits are
        # stream-side), so a window's event never covers a later window's decode, and a later
        # window's collectives (rows it ships) are stream-ordered after this scatter.
        for w in self.queue:
            if w.done:
                continue
            if w.work is None:
                if not w.future.done():
                    break
                if any(not sw.done for sw in w.ship_src.values()):
                    break   # a row it ships is still being delivered here: its ok flag is not final
                w.store._issue(w, rank, world, w.future.result(), comm, stream)
                if w.store.device.type == "cuda":
                    w.store._finish(w, world, stream)
            if not w.done and w.store.device.type != "cuda":
                break   # host arenas scatter at the finish: a later window may ship these rows
        while self.queue:
            w = self.queue[0]
            if not w.done and (w.work is None or not w.store._finish(w, world, stream)):
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
