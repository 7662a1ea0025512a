"""Elastic process group: epoch-versioned communicators rebuilt over survivors.

RCCL is not elastic — a rank that dies mid-collective hangs its peers (SURVEY
§7.4 item 3). The recovery protocol here:

 * the rendezvous store is a ``FileStore`` on the node's local filesystem (one
   node = one filesystem; 8 GPUs per MI355X node), so NO rank hosts it: any rank,
   the coordinator included, can die without taking the rendezvous with it (the
   previous TCPStore lived inside global rank 0). A TCPStore host can still be
   given for multi-node runs (``store_host``), at the price of that single host;
 * communicator *epoch e* is initialised through ``PrefixStore("epoch<e>")`` over
   the epoch's member list;
 * liveness comes from the host-side SWIM detector (cluster/), never from the
   collective library; collectives are issued ``async_op=True`` and polled
   (``Work.is_completed``), so a rank declared dead while a collective is pending
   makes the survivors ABORT the communicator (``_abort_process_group``: on RCCL
   this is ncclCommAbort, which also releases the collective kernels still queued
   on RCCL's own stream) instead of hanging. The host never calls ``Work.wait``
   before the poll has seen completion, so no compute stream is ever ordered
   behind a collective that will not finish;
 * agreement on the next member list: every survivor proposes its own survivor
   view with ``compare_set(members<e+1>)`` — the first proposal wins, everyone
   adopts it (a rank not in it leaves), then joins epoch e+1 with its new rank.

Works identically on gloo (CPU tests) and nccl (= RCCL on ROCm).
"""
from __future__ import annotations

import datetime
import hashlib
import json
import logging
import os
import time
from typing import List, Optional, Set

import numpy as np
import torch
import torch.distributed as dist
from torch.distributed import distributed_c10d as c10d

log = logging.getLogger(__name__)


class CollectiveFailure(RuntimeError):
    """A collective could not complete (peer died / communicator aborted)."""


class ShmExchange:
    """The per-step control exchange over node-local shared memory
    (csrc/host/shm_exchange.cpp, libdml_host.so): all-gather semantics for a fixed-size
    int64 record, waited for in native code with the GIL released. ``poll()`` is called
    every ``slice_us`` while waiting; it raises CollectiveFailure when the failure
    detector has confirmed a member dead (a dead rank never publishes)."""

    REC_CAP = 32768

    def __init__(self, name: str, world: int, rank: int):
        import ctypes as C

        from ..serving.output import _host_lib

        L = _host_lib()
        if L is None:
            raise CollectiveFailure("shared-memory exchange needs libdml_host.so")
        L.dml_shm_open.restype = C.c_void_p
        L.dml_shm_open.argtypes = [C.c_char_p, C.c_int, C.c_int]
        L.dml_shm_exchange.restype = C.c_int
        L.dml_shm_exchange.argtypes = [C.c_void_p, C.c_int, C.c_longlong, C.c_void_p, C.c_int, C.c_void_p, C.c_int]
        L.dml_shm_close.restype = None
        L.dml_shm_close.argtypes = [C.c_void_p, C.c_int]
        self.L, self.name, self.world, self.rank = L, name, world, rank
        self.h = L.dml_shm_open(name.encode(), world, self.REC_CAP)
        if not self.h:
            raise CollectiveFailure(f"shm_open({name}) failed")
        self.step = 0

    def exchange(self, out, t, poll, timeout_s: float = 120.0, slice_us: int = 2000) -> None:
        """``t`` / ``out``: contiguous CPU torch tensors or numpy arrays (numpy: no torch call,
        so no GIL hand-off to the rank's other threads on the serve loop's path)."""
        if isinstance(t, np.ndarray):
            nb, src, dst = t.nbytes, t.ctypes.data, out.ctypes.data
            ok = t.flags.c_contiguous and out.flags.c_contiguous
        else:
            nb, src, dst = t.numel() * t.element_size(), t.data_ptr(), out.data_ptr()
            ok = t.is_contiguous() and out.is_contiguous() and t.device.type == "cpu"
        if nb > self.REC_CAP or not ok:
            raise CollectiveFailure("shm exchange: record too large or not a contiguous CPU buffer")
        self.step += 1
        t0 = time.monotonic()
        while True:
            rc = self.L.dml_shm_exchange(self.h, self.rank, self.step, src, nb, dst, slice_us)
            if rc == 0:
                return
            if rc < 0:
                raise CollectiveFailure("shm exchange: bad arguments")
            poll()
            if time.monotonic() - t0 > timeout_s:
                raise CollectiveFailure("shm exchange timeout")

    def close(self, unlink: bool = False) -> None:
        if self.h:
            self.L.dml_shm_close(self.h, int(unlink))
            self.h = None


def shm_tag(store_path: str) -> str:
    """The per-rendezvous prefix of the shared-memory segment names (/dev/shm/dml_<tag>_...)."""
    return hashlib.sha1(os.path.abspath(store_path).encode()).hexdigest()[:12]


def unlink_stale_segments(store_path: str) -> int:
    """Remove every shared-memory exchange segment of a rendezvous path (the launcher calls
    this when it (re)creates the path: segments of a killed previous run never unlinked
    themselves). Returns how many were removed."""
    pre = f"dml_{shm_tag(store_path)}_"
    n = 0
    try:
        names = os.listdir("/dev/shm")
    except OSError:
        return 0
    for f in names:
        if f.startswith(pre):
            try:
                os.unlink(os.path.join("/dev/shm", f))
                n += 1
            except OSError:
                pass
    return n


def default_store_path(tag: str) -> str:
    base = os.environ.get("DML_RDZV_DIR", "/tmp")
    return os.path.join(base, f"dml_rdzv_{tag}")


class ElasticGroup:
    def __init__(self, global_rank: int, world: int, store_path: Optional[str] = None, backend: str = "gloo",
                 device: Optional[torch.device] = None, timeout_s: float = 60.0, store_host: Optional[str] = None,
                 store_port: int = 0, data_backend: Optional[str] = None, join: bool = False,
                 join_timeout_s: float = 300.0, shm_exchange: bool = False):
        """``backend``: the default group (control collectives); ``data_backend``:
        a second group over the same members for bulk tensors (e.g. control on
        host gloo, decoded images on RCCL), rebuilt with every epoch.
        ``join``: this process RE-joins a running job (a restarted rank): it
        waits until the coordinator admits it into a new epoch (``admit``).
        ``shm_exchange``: ``exchange`` (the service's per-step control collective) runs
        over node-local shared memory (ShmExchange), one segment per epoch, instead of
        the default group — the ranks must share a node (the FileStore already implies it)."""
        self.grank, self.backend, self.device = global_rank, backend, device
        self.data_backend = data_backend or backend
        self.data_group = None
        self.result_group = None
        self._graveyard: list = []
        self.members: List[int] = list(range(world))
        self.prev_members: List[int] = list(self.members)   # the member list of the previous epoch
        self.epoch = 0
        self.timeout = datetime.timedelta(seconds=timeout_s)
        if store_host is not None:  # multi-node: a TCPStore on one host (that host is then a SPOF)
            self.store = dist.TCPStore(store_host, store_port, world_size=None, is_master=(global_rank == 0),
                                       timeout=self.timeout, wait_for_workers=False)
        else:
            if store_path is None:
                raise ValueError("ElasticGroup needs a store_path (FileStore) or a store_host")
            self.store = dist.FileStore(store_path, -1)
            self.store.set_timeout(self.timeout)
        self.dead: Set[int] = set()          # fed by the failure detector (thread-safe set ops)
        self.joiners: Set[int] = set()       # ranks alive again but outside the group (SWIM rejoin)
        self.aborts = 0
        self._moved_t, self._moved_every_s = 0.0, 0.05
        self.shm_exchange = shm_exchange and store_host is None
        self._shm: Optional[ShmExchange] = None
        self._shm_names: List[str] = []
        # the same name in every rank process (str hash() is salted per process) AND unique per
        # job: a rank that was SIGKILLed never unlinks its segments, so a relaunch over a reused
        # --rdzv path would otherwise open the old segment, whose per-rank step counters are
        # still high, and apply the previous run's records as this step's. The
        # first rank to reach the store fixes a random nonce (compare_set); every other rank
        # and every later joiner of this store reads that one.
        self._shm_tag = shm_tag(store_path or "") + "_" + self._job_nonce()
        if join:
            self._await_admission(join_timeout_s)
        self._init_pg()

    def _job_nonce(self) -> str:
        mine = os.urandom(6).hex()
        return self.store.compare_set("shm_nonce", "", mine).decode()

    # --------------------------------------------------------------- group --
    @property
    def rank(self) -> int:
        return self.members.index(self.grank)

    @property
    def world(self) -> int:
        return len(self.members)

    def group_rank_of(self, grank: int) -> int:
        return self.members.index(grank)

    def _init_pg(self) -> None:
        prefix = dist.PrefixStore(f"epoch{self.epoch}", self.store)
        kw = {}
        if self.backend == "nccl" and self.device is not None:
            kw["device_id"] = self.device
        dist.init_process_group(self.backend, store=prefix, rank=self.rank, world_size=self.world,
                                timeout=self.timeout, **kw)
        # the image windows' all-gathers always get a group of their own: they are issued
        # when a window's decode finishes, which is not ordered against the step's control
        # exchange across ranks (gloo / RCCL match collectives by issue order per group)
        self.data_group = dist.new_group(list(range(self.world)), backend=self.data_backend)
        # the service's per-step result gather (top-5 rows -> the coordinator) on a group of its
        # own too: it is issued at the same step on every rank, the windows' collectives are not
        self.result_group = dist.new_group(list(range(self.world)), backend=self.data_backend)
        if self.shm_exchange:
            if self._shm is not None:
                self._shm.close()
            name = f"/dml_{self._shm_tag}_e{self.epoch}_" + "-".join(map(str, self.members))
            self._shm_names.append(name)
            self._shm = ShmExchange(name, self.world, self.rank)
        log.info("rank %d joined epoch %d (%d members)", self.grank, self.epoch, self.world)

    def _teardown(self, abort: bool) -> None:
        """End the current communicator. ``abort``: a collective may still be
        pending (a peer died) — abort it explicitly (RCCL: ncclCommAbort) so
        nothing waits on it, then destroy the group."""
        if not dist.is_initialized():
            return
        self.data_group = None
        self.result_group = None
        if abort:
            # every group of the epoch (RCCL: ncclCommAbort; gloo: closes the pairs, so an
            # image window's all-gather still pending on a peer that went on to rebuild
            # fails at once instead of holding destroy_process_group for the timeout)
            # the aborted groups stay referenced: the last reference dropping inside the abort
            # would run the gloo group's destructor there, which joins its worker threads
            # behind ops of the failed epoch (observed: minutes inside the abort). Only the
            # last aborted epoch's groups are kept: the ones before it were released at the
            # previous abort's end, once no op of theirs could still be queued (their epoch's
            # successor ran whole steps since), so kills and rejoins do not accumulate gloo
            # threads / sockets / RCCL communicators over a long-running service
            old = self._graveyard
            self._graveyard = list(c10d._world.pg_map.keys())
            c10d._abort_process_group()
            del old
            self.aborts += 1
            return  # the abort destroyed the default group
        try:
            dist.destroy_process_group()
        except Exception as e:  # gloo: a dead peer's socket may already be closed
            log.debug("destroy_process_group: %s", e)

    # -------------------------------------------------------- collectives --
    def wait(self, work, poll_s: float = 0.0002) -> None:
        """Wait for an async collective, aborting if a member is declared dead.

        gloo: a blocking wait (GIL released). A dead peer's closed sockets fail
        the collective on every survivor at once, and polling from Python costs
        the gloo threads their CPU: at world 8 on 8 cores an all-gather took
        1.9 ms blocking vs 8-12 ms polled (yield or spin). nccl (RCCL) cannot
        report a dead peer, so it is polled against the SWIM verdicts."""
        if self.backend == "gloo":
            # a blocking wait (GIL released). A sliced wait (gloo raises "timed out" at the
            # slice end) left multi-hop collectives broken on the ranks that sliced; the
            # service's per-step exchange polls the SWIM verdicts on the shared-memory path
            # instead (ShmExchange), so a hung-but-connected peer no longer stalls the loop
            try:
                work.wait()
            except Exception as e:  # gloo raises when a peer's socket closes / on its timeout
                raise CollectiveFailure(str(e)) from e
            return
        t0 = time.monotonic()
        while not work.is_completed():
            if self.dead & set(self.members):
                raise CollectiveFailure(f"members {sorted(self.dead & set(self.members))} declared dead")
            if time.monotonic() - t0 > self.timeout.total_seconds():
                raise CollectiveFailure("collective timeout")
            time.sleep(poll_s)
        try:
            work.wait()
        except Exception as e:  # gloo raises when a peer's socket closes
            raise CollectiveFailure(str(e)) from e

    def _poll_dead(self) -> None:
        """(between shared-memory wait slices) a member SWIM confirmed dead fails the exchange;
        so does a next epoch the others fixed WITHOUT this rank (a live rank they declared
        dead — a false suspicion — would otherwise wait out the whole timeout on a segment
        nobody else writes any more; a next epoch that holds this rank is a growth, announced
        by this very exchange). The store is looked at every ``_moved_every_s``."""
        if self.dead & set(self.members):
            raise CollectiveFailure(f"members {sorted(self.dead & set(self.members))} declared dead")
        now = time.monotonic()
        if now - self._moved_t >= self._moved_every_s:
            self._moved_t = now
            key = f"members{self.epoch + 1}"
            if self.store.check([key]) and self.grank not in json.loads(self.store.get(key).decode()):
                raise CollectiveFailure(f"removed from the group: epoch {self.epoch + 1} fixed without this rank")

    def _run(self, fn, *args, **kw) -> None:
        try:
            w = fn(*args, async_op=True, **kw)
        except Exception as e:
            raise CollectiveFailure(str(e)) from e
        self.wait(w)

    def broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        """``src`` is a GROUP rank."""
        self._run(dist.broadcast, t, src=src)

    def broadcast_bytes(self, data: Optional[bytes], n: int, src: int = 0) -> bytes:
        """Broadcast ``n`` bytes (the service's log records; ``data`` on GROUP rank ``src``)
        and return them on every rank. With the shared-memory exchange they go through that
        segment in record-sized chunks (numpy, no torch call), waited for with the same
        dead-member / moved-epoch polling as the step's exchange (a gloo broadcast blocks
        without either: a peer that left mid-broadcast held this rank for the full
        collective timeout)."""
        if self._shm is None:
            t = torch.zeros(n, dtype=torch.uint8, device=self.device if self.backend == "nccl" else "cpu")
            if self.rank == src:
                t.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
            self.broadcast(t, src=src)
            return data if self.rank == src else bytes(t.cpu().numpy())
        cap = ShmExchange.REC_CAP
        mine = np.frombuffer(data, np.uint8) if self.rank == src else None
        got = bytearray(n) if self.rank != src else None
        out = np.empty((self.world, min(cap, max(n, 1))), np.uint8)
        zeros = np.zeros(min(cap, max(n, 1)), np.uint8)
        for o in range(0, n, cap):
            k = min(cap, n - o)
            chunk = np.ascontiguousarray(mine[o:o + k]) if mine is not None else zeros[:k]
            ob = out if k == out.shape[1] else np.empty((self.world, k), np.uint8)
            self._shm.exchange(ob, chunk, self._poll_dead, self.timeout.total_seconds())
            if got is not None:
                got[o:o + k] = ob[src].tobytes()
        return data if got is None else bytes(got)

    def gather(self, t: torch.Tensor, bufs: Optional[List[torch.Tensor]], dst: int = 0) -> None:
        self._run(dist.gather, t, bufs if self.rank == dst else None, dst=dst)

    def all_gather(self, bufs: List[torch.Tensor], t: torch.Tensor) -> None:
        self._run(dist.all_gather, bufs, t)

    def all_gather_into(self, out: torch.Tensor, t: torch.Tensor) -> None:
        """out = concat of every rank's t along dim 0 (out: [world * t.shape[0], ...]
        or [world, *t.shape])."""
        if self.backend == "nccl":
            self._run(dist.all_gather_into_tensor, out, t)
        else:
            self._run(dist.all_gather, list(out.view(self.world, *t.shape).unbind(0)), t)

    def exchange(self, out, t, root: int) -> None:
        """out[r] = rank r's t on every rank (all-gather semantics; ``root`` a
        GROUP rank). gloo: a gather to ``root`` plus a broadcast from it - two
        hops instead of a ring's world-1 (world 8 on 8 cores: 0.54 ms vs 2.1 ms
        for a 1.7 KB record); nccl: the ring all-gather. numpy buffers: the
        shared-memory exchange only (the service's CPU path)."""
        if self._shm is not None and (isinstance(t, np.ndarray) or t.device.type == "cpu"):
            self._shm.exchange(out, t, self._poll_dead, self.timeout.total_seconds())
            return
        if isinstance(t, np.ndarray):
            tt, ot = torch.from_numpy(t), torch.from_numpy(out)
            self.exchange(ot, tt, root)
            return
        if self.backend != "gloo":
            self.all_gather_into(out, t)
            return
        self._run(dist.gather, t, list(out.view(self.world, *t.shape).unbind(0)) if self.rank == root else None,
                  dst=root)
        self._run(dist.broadcast, out, src=root)

    def all_gather_data(self, out: torch.Tensor, t: torch.Tensor) -> None:
        """all-gather on the data group (bulk tensors): out = concat of every
        rank's t along dim 0 (all_gather_into_tensor semantics)."""
        if self.data_backend == "nccl":
            self._run(dist.all_gather_into_tensor, out, t, group=self.data_group)
        else:
            self._run(dist.all_gather, list(out.view(self.world, *t.shape).unbind(0)), t, group=self.data_group)

    def all_gather_data_async(self, out: torch.Tensor, t: torch.Tensor):
        """Issue the data-group all-gather without waiting; returns the Work (RCCL: wait()
        makes the current stream wait for it; gloo: poll is_completed()). The caller
        issues these in the same order on every rank."""
        try:
            if self.data_backend == "nccl":
                return dist.all_gather_into_tensor(out, t, group=self.data_group, async_op=True)
            return dist.all_gather(list(out.view(self.world, *t.shape).unbind(0)), t, group=self.data_group,
                                   async_op=True)
        except Exception as e:
            raise CollectiveFailure(str(e)) from e

    def all_to_all_data_async(self, out: torch.Tensor, t: torch.Tensor, out_splits: List[int],
                              in_splits: List[int]):
        """Issue an uneven all-to-all on the data group (rows of dim 0: ``in_splits[r]``
        rows of ``t`` go to group rank r, ``out_splits[s]`` rows arrive from s); returns the
        Work (same contract as all_gather_data_async)."""
        try:
            return dist.all_to_all_single(out, t, out_splits, in_splits, group=self.data_group, async_op=True)
        except Exception as e:
            raise CollectiveFailure(str(e)) from e

    def all_reduce_data_async(self, t: torch.Tensor):
        """Issue a SUM all-reduce on the data group; returns the Work."""
        try:
            return dist.all_reduce(t, group=self.data_group, async_op=True)
        except Exception as e:
            raise CollectiveFailure(str(e)) from e

    def gather_result(self, t: torch.Tensor, outs: Optional[List[torch.Tensor]], dst: int) -> None:
        """gather on the result group (RCCL on a GPU node): ``outs`` (on ``dst`` only) <- every
        rank's ``t``; ``dst`` is a GROUP rank."""
        self._run(dist.gather, t, outs if self.rank == dst else None, dst=dst, group=self.result_group)

    def gather_result_async(self, t, outs, dst):
        """The result gather, not waited for (the service polls ``is_completed``); the
        epoch's result group orders it against the other result gathers only."""
        try:
            return dist.gather(t, outs if self.rank == dst else None, dst=dst, group=self.result_group,
                               async_op=True)
        except Exception as e:
            raise CollectiveFailure(str(e)) from e

    def broadcast_data(self, t: torch.Tensor, src: int = 0) -> None:
        """broadcast on the data group (bulk tensors); ``src`` is a GROUP rank."""
        self._run(dist.broadcast, t, src=src, group=self.data_group)

    def barrier(self) -> None:
        t = torch.zeros(1, device=self.device if self.backend == "nccl" else "cpu")
        self._run(dist.all_reduce, t)

    # ------------------------------------------------------------ rebuild --
    def rebuild(self, dead: Set[int], decide: bool = True) -> List[int]:
        """Move to epoch+1 over the survivors. Every survivor proposes its view
        of the member list; the first proposal in the store wins (compare-set),
        so all survivors adopt the same list without a designated decider."""
        nxt = self.epoch + 1
        key = f"members{nxt}"
        mine = [m for m in self.members if m not in dead]
        won = self.store.compare_set(key, "", json.dumps(mine))
        members = json.loads(won)
        for d in set(self.members) - set(members):  # a stale admission must not lure a restarted rank back
            try:
                self.store.delete_key(f"admit{d}")
            except Exception:
                pass
        self._teardown(abort=True)
        if self.grank not in members:
            raise CollectiveFailure("this rank was removed from the group")
        self.prev_members, self.members = self.members, members
        self.epoch = nxt
        self.dead.intersection_update(self.members)  # forget the removed ranks
        try:
            self._init_pg()
        except Exception as e:
            # the agreed list held a rank that never arrived (a second failure SWIM
            # had not confirmed when the list was fixed): the caller rebuilds again
            # at epoch+1 with the dead set it has learned since
            try:
                dist.destroy_process_group()
            except Exception:
                pass
            raise CollectiveFailure(f"epoch {nxt} initialisation failed: {e}") from e
        return members

    # ------------------------------------------------------------- growth --
    def admit(self, joiners: Set[int]) -> List[int]:
        """(coordinator) Propose epoch e+1 = members + joiners and tell each
        joiner which epoch to join. Returns the proposed member list (the list
        that compare_set fixed: a concurrent failure rebuild may win instead)."""
        nxt = self.epoch + 1
        want = sorted(set(self.members) | set(joiners))
        won = json.loads(self.store.compare_set(f"members{nxt}", "", json.dumps(want)))
        for g in joiners:
            if g in won:
                self.store.set(f"admit{g}", str(nxt))
        return won

    def grow(self, members: List[int]) -> List[int]:
        """Every current member: move to epoch e+1 over ``members``. The list is the one
        in the store, so every member and the joiners agree on it. The old groups are
        aborted, not destroyed: no control collective is pending at a step boundary, but an
        image window's data-group all-gather may be — issued here, not yet by a peer whose
        decode was still running, and dropped by every rank at this boundary (measured: a
        destroy waited out the 30 s gloo timeout behind it while the others' init of the
        new epoch timed out)."""
        nxt = self.epoch + 1
        won = json.loads(self.store.compare_set(f"members{nxt}", "", json.dumps(sorted(members))))
        self._teardown(abort=True)
        if self.grank not in won:
            raise CollectiveFailure("this rank was removed from the group")
        self.prev_members, self.members = self.members, won
        self.epoch = nxt
        self.dead.intersection_update(self.members)
        self.joiners.difference_update(self.members)
        self._init_pg()
        return won

    def rejoin(self, timeout_s: float) -> List[int]:
        """A live rank the others removed (a false suspicion: it was slow, not dead) joins
        again like a restarted one: it waits for its admission into a later epoch (the
        coordinator admits it once SWIM sees it alive) and initialises that epoch."""
        self._teardown(abort=True)
        self.dead.clear()
        self._await_admission(timeout_s, after=self.epoch)
        self._init_pg()
        return self.members

    def _await_admission(self, timeout_s: float, after: int = -1) -> None:
        """(joiner) Wait for ``admit<g>`` = the epoch whose member list holds
        this rank, then take that epoch's member list from the store."""
        key = f"admit{self.grank}"
        t0 = time.monotonic()
        while True:
            if self.store.check([key]):
                e = int(self.store.get(key).decode())
                members = json.loads(self.store.get(f"members{e}").decode())
                if self.grank in members and e > after:
                    prev = self.store.get(f"members{e - 1}").decode() if e > 0 else json.dumps(members)
                    self.prev_members = json.loads(prev)
                    self.epoch, self.members = e, members
                    log.info("rank %d admitted into epoch %d", self.grank, e)
                    return
            if time.monotonic() - t0 > timeout_s:
                raise CollectiveFailure("not admitted into the job")
            time.sleep(0.05)

    def close(self) -> None:
        self._teardown(abort=False)
        if self._shm is not None:
            self._shm.close()
            self._shm = None
        for name in self._shm_names:  # every epoch's segment (ranks that died never unlink theirs)
            try:
                os.unlink("/dev/shm" + name)
            except OSError:
                pass
