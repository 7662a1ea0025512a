"""Elastic process group: epoch-versioned communicators rebuilt over survivors.

RCCL is not elastic — a rank that dies mid-collective hangs its peers (SURVEY
§7.4 item 3). The recovery protocol here:

 * a persistent TCPStore hosted by global rank 0 (the coordinator) outlives
   every communicator; communicator *epoch e* is initialised through
   ``PrefixStore("epoch<e>", store)`` over the current member list;
 * liveness comes from the host-side SWIM detector (cluster/), never from the
   collective library; collectives are issued ``async_op=True`` and polled, so
   a rank declared dead while a collective is pending makes the survivors
   ``abort()`` the communicator instead of hanging;
 * the coordinator publishes the survivor list for epoch e+1 in the store; every
   survivor reads it, tears down epoch e and joins epoch e+1 with its new rank.

Works identically on gloo (CPU tests) and nccl (= RCCL on ROCm).
"""
from __future__ import annotations

import datetime
import json
import logging
import os
import time
from typing import Callable, List, Optional, Set

import torch
import torch.distributed as dist

log = logging.getLogger(__name__)


class CollectiveFailure(RuntimeError):
    """A collective could not complete (peer died / communicator aborted)."""


class ElasticGroup:
    def __init__(self, global_rank: int, world: int, host: str = "127.0.0.1", port: int = 29555,
                 backend: str = "gloo", device: Optional[torch.device] = None, timeout_s: float = 60.0):
        self.grank, self.backend, self.device = global_rank, backend, device
        self.members: List[int] = list(range(world))
        self.epoch = 0
        self.timeout = datetime.timedelta(seconds=timeout_s)
        self.store = dist.TCPStore(host, port, world_size=None, is_master=(global_rank == 0),
                                   timeout=self.timeout, wait_for_workers=False)
        self.dead: Set[int] = set()          # fed by the failure detector (thread-safe set ops)
        self._init_pg()

    # --------------------------------------------------------------- group --
    @property
    def rank(self) -> int:
        return self.members.index(self.grank)

    @property
    def world(self) -> int:
        return len(self.members)

    def _init_pg(self) -> None:
        prefix = dist.PrefixStore(f"epoch{self.epoch}", self.store)
        kw = {}
        if self.backend == "nccl" and self.device is not None:
            kw["device_id"] = self.device
        dist.init_process_group(self.backend, store=prefix, rank=self.rank, world_size=self.world,
                                timeout=self.timeout, **kw)
        log.info("rank %d joined epoch %d (%d members)", self.grank, self.epoch, self.world)

    def _teardown(self) -> None:
        try:
            pg = dist.group.WORLD
            if pg is not None and hasattr(pg, "abort"):
                pg.abort()
        except Exception:  # pragma: no cover - best effort
            pass
        try:
            dist.destroy_process_group()
        except Exception:  # pragma: no cover
            pass

    # -------------------------------------------------------- collectives --
    def wait(self, work, poll_s: float = 0.0002) -> None:
        """Wait for an async collective, aborting if a member is declared dead."""
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

    def broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        try:
            w = dist.broadcast(t, src=src, async_op=True)
        except Exception as e:
            raise CollectiveFailure(str(e)) from e
        self.wait(w)

    def gather(self, t: torch.Tensor, bufs: Optional[List[torch.Tensor]]) -> None:
        try:
            w = dist.gather(t, bufs if self.rank == 0 else None, dst=0, async_op=True)
        except Exception as e:
            raise CollectiveFailure(str(e)) from e
        self.wait(w)

    # ------------------------------------------------------------ rebuild --
    def rebuild(self, dead: Set[int], decide: bool) -> None:
        """Move to epoch+1 over the survivors. The coordinator (``decide=True``)
        publishes the member list; everyone else reads it from the store."""
        nxt = self.epoch + 1
        key = f"members{nxt}"
        if decide:
            members = [m for m in self.members if m not in dead]
            self.store.set(key, json.dumps(members))
        else:
            self.store.wait([key], self.timeout)
            members = json.loads(self.store.get(key))
        self._teardown()
        if self.grank not in members:
            raise CollectiveFailure("this rank was removed from the group")
        self.members = members
        self.epoch = nxt
        self.dead.intersection_update(self.members)  # forget the removed ranks
        self._init_pg()

    def close(self) -> None:
        self._teardown()
