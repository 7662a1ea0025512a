"""SWIM failure detector driver (asyncio) over a control-plane Endpoint.

Reference (worker.py:1083-1199): every PING_DURATION (12 s shipped / 2.5 s in
the README) ping the 3 ring targets with the full membership list, wait
PING_TIMEOUT for an ACK, suspect after > 3 consecutive misses; no indirect
probes. Detection took ~76-100 s with the shipped constants.

Here: each period probe the ring targets concurrently; on a missed ACK ask
``indirect_k`` other members to PING_REQ the target (so one lossy link does not
cause a false suspicion); suspect after ``misses_to_suspect`` failed rounds;
suspicion is disseminated by gossip and confirmed DEAD by the membership timer
unless refuted. Every PING/ACK/PING_REQ carries the membership digest. Default
timings are sub-second for the single-node GPU deployment (loopback RTT ~50 us).
"""
from __future__ import annotations

import asyncio
import logging
import random
from typing import Dict, Optional

from .frames import Frame, MsgType
from .membership import MembershipList, Status
from .transport import Endpoint

log = logging.getLogger(__name__)


class FailureDetector:
    def __init__(self, ep: Endpoint, ml: MembershipList, period: float = 0.5, ping_timeout: float = 0.25,
                 indirect_k: int = 2, misses_to_suspect: int = 1, seed: int = 0):
        self.ep, self.ml = ep, ml
        self.period, self.ping_timeout = period, ping_timeout
        self.indirect_k, self.misses_to_suspect = indirect_k, misses_to_suspect
        self.rng = random.Random(seed)
        self.misses: Dict[str, int] = {}
        self.enabled = True  # menu option 4 ("leave") disables probing and acking
        self.rounds = 0
        ep.on(MsgType.PING, self._on_ping)
        ep.on(MsgType.INTRODUCE, self._on_ping)
        ep.on(MsgType.PING_REQ, self._on_ping_req)
        ep.on(MsgType.LEAVE, self._on_leave)
        self._task: Optional[asyncio.Task] = None

    # -------------------------------------------------------------- handlers --
    def _absorb(self, fr: Frame) -> None:
        d = fr.payload.get("members")
        if d:
            self.ml.merge(d)

    async def _on_ping(self, fr: Frame) -> None:
        if not self.enabled:
            return
        self._absorb(fr)
        self.ml.mark_alive(fr.sender, fr.payload.get("inc"))
        await self.ep.reply(fr, MsgType.ACK, {"members": self.ml.digest(), "inc": self.ml.me.incarnation})

    async def _on_ping_req(self, fr: Frame) -> None:
        if not self.enabled:
            return
        self._absorb(fr)
        target = fr.payload["target"]
        ok = await self._ping(target)
        await self.ep.reply(fr, MsgType.PING_REQ_ACK, {"target": target, "ok": ok, "members": self.ml.digest()})

    async def _on_leave(self, fr: Frame) -> None:
        self._absorb(fr)

    # ---------------------------------------------------------------- probes --
    async def _ping(self, target: str) -> bool:
        r = await self.ep.request(target, MsgType.PING, {"members": self.ml.digest(), "inc": self.ml.me.incarnation},
                                  timeout=self.ping_timeout)
        if r is None:
            return False
        self._absorb(r)
        self.ml.mark_alive(target, r.payload.get("inc"))
        return True

    async def probe(self, target: str) -> bool:
        if await self._ping(target):
            self.misses[target] = 0
            return True
        helpers = [m for m in self.ml.alive(include_self=False) if m != target]
        self.rng.shuffle(helpers)
        helpers = helpers[: self.indirect_k]
        if helpers:
            reqs = [self.ep.request(h, MsgType.PING_REQ, {"target": target, "members": self.ml.digest()},
                                    timeout=2 * self.ping_timeout) for h in helpers]
            for r in await asyncio.gather(*reqs):
                if r is not None:
                    self._absorb(r)
                    if r.payload.get("ok"):
                        self.misses[target] = 0
                        self.ml.mark_alive(target)
                        return True
        self.misses[target] = self.misses.get(target, 0) + 1
        if self.misses[target] >= self.misses_to_suspect:
            m = self.ml.get(target)
            if m is not None and m.status == Status.ALIVE:
                log.info("%s suspects %s", self.ml.self_name, target)
                self.ml.suspect(target)
        return False

    async def round(self) -> None:
        self.rounds += 1
        self.ml.tick()
        if not self.enabled:
            return
        targets = self.ml.ring_targets()
        if targets:
            await asyncio.gather(*(self.probe(t) for t in targets))
        self.ml.tick()

    async def run(self) -> None:
        while True:
            await self.round()
            await asyncio.sleep(self.period)

    def start(self) -> asyncio.Task:
        self._task = asyncio.get_running_loop().create_task(self.run())
        return self._task

    def stop(self) -> None:
        if self._task:
            self._task.cancel()

    async def leave(self) -> None:
        """Graceful leave: tell the ring, then stop probing/acking."""
        self.enabled = False  # before ml.leave(): a round() in between must not probe from a LEFT self
        self.ml.leave()
        for t in self.ml.alive(include_self=False):
            await self.ep.send(t, MsgType.LEAVE, {"members": self.ml.digest()})

    async def join(self, introducer: str, timeout: float = 1.0, retries: int = 3) -> bool:
        """INTRODUCE to a known member (the leader / introducer) and merge its list."""
        r = await self.ep.request(introducer, MsgType.INTRODUCE, {"members": self.ml.digest(),
                                                                  "inc": self.ml.me.incarnation},
                                  timeout=timeout, retries=retries)
        if r is None:
            return False
        self._absorb(r)
        return True
