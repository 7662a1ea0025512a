"""Leader election: bully algorithm over the alive coordinator-eligible nodes.

Reference (election.py:7-32, worker.py:621-649, 1161-1178): when the leader is
removed every node floods ELECTION to its ping targets, and the winner is
hard-coded — ``check_if_leader`` is true only on host H2, so if H2 is also dead
nobody can ever win (election.py:27).

Here: priority = (standby flag, node name) over members whose meta says
``eligible``; a node sends ELECTION to every higher-priority alive node, and if
none answers ELECTION_OK within ``timeout`` it becomes leader and broadcasts
COORDINATE. A node that receives ELECTION from a lower-priority node answers
ELECTION_OK and runs its own election. Followers answer COORDINATE with
COORDINATE_ACK carrying whatever ``ack_payload()`` returns (the reference sends
its local file list so the new leader can rebuild the SDFS map), and the new
leader hands all ACKs to ``on_elected``. Non-eligible nodes (GPU workers) only
follow.
"""
from __future__ import annotations

import asyncio
import logging
from typing import Callable, Dict, List, Optional, Tuple

from .frames import Frame, MsgType
from .membership import MembershipList
from .transport import Endpoint

log = logging.getLogger(__name__)


class Election:
    def __init__(self, ep: Endpoint, ml: MembershipList, timeout: float = 0.5,
                 ack_payload: Optional[Callable[[], dict]] = None,
                 on_elected: Optional[Callable[[Dict[str, dict]], None]] = None,
                 on_new_leader: Optional[Callable[[str], None]] = None):
        self.ep, self.ml, self.timeout = ep, ml, timeout
        self.leader: Optional[str] = None
        self.in_election = False
        self.ack_payload = ack_payload or (lambda: {})
        self.on_elected = on_elected
        self.on_new_leader = on_new_leader
        self._ok = asyncio.Event()
        self._coord = asyncio.Event()
        self.elections_won = 0
        self._task: Optional[asyncio.Task] = None
        # test hook: a fail-over election (the leader died) starts this much later, so the
        # service outruns the store-leader election deterministically (tests/test_elastic_service.py)
        self.failover_delay_s = 0.0
        ep.on(MsgType.ELECTION, self._on_election)
        ep.on(MsgType.ELECTION_OK, self._on_ok)
        ep.on(MsgType.COORDINATE, self._on_coordinate)

    # ---------------------------------------------------------- priority --
    def eligible(self, name: str) -> bool:
        m = self.ml.get(name)
        return m is not None and bool(m.meta.get("eligible"))

    def priority(self, name: str) -> Tuple[int, int, str]:
        """(standby flag, numeric ``prio`` meta, name): the RCCL service's rank
        nodes carry prio = global rank, so the highest alive rank leads — the
        same rank the collective service picks as its coordinator."""
        m = self.ml.get(name)
        standby = 1 if (m is not None and m.meta.get("role") == "standby") else 0
        prio = int(m.meta.get("prio", 0)) if m is not None else 0
        return standby, prio, name

    def candidates(self) -> List[str]:
        return sorted((n for n in self.ml.alive() if self.eligible(n)), key=self.priority, reverse=True)

    # ---------------------------------------------------------- protocol --
    def leader_failed(self, name: str) -> None:
        if name == self.leader:
            log.info("%s: leader %s failed -> election", self.ml.self_name, name)
            self.leader = None
            self.trigger()

    def trigger(self) -> None:
        if self._task is None or self._task.done():
            self._task = asyncio.get_running_loop().create_task(self.run_election())

    async def run_election(self) -> Optional[str]:
        me = self.ml.self_name
        self.in_election = True
        try:
            if self.failover_delay_s > 0 and self.leader is None:
                await asyncio.sleep(self.failover_delay_s)
            for _ in range(5):
                if not self.eligible(me):
                    # followers just poke the best candidate and wait for COORDINATE
                    cands = self.candidates()
                    if cands:
                        self._coord.clear()
                        await self.ep.send(cands[0], MsgType.ELECTION, {})
                        try:
                            await asyncio.wait_for(self._coord.wait(), 4 * self.timeout)
                            return self.leader
                        except asyncio.TimeoutError:
                            continue
                    return None
                higher = [n for n in self.candidates() if self.priority(n) > self.priority(me)]
                self._ok.clear()
                self._coord.clear()
                for h in higher:
                    await self.ep.send(h, MsgType.ELECTION, {})
                if higher:
                    try:
                        await asyncio.wait_for(self._ok.wait(), self.timeout)
                        # someone higher is alive: wait for its COORDINATE
                        await asyncio.wait_for(self._coord.wait(), 4 * self.timeout)
                        return self.leader
                    except asyncio.TimeoutError:
                        if self._coord.is_set():
                            return self.leader
                        if self._ok.is_set():
                            continue  # higher node stalled: retry
                await self._become_leader()
                return me
            return self.leader
        finally:
            self.in_election = False

    async def _become_leader(self) -> None:
        me = self.ml.self_name
        self.leader = me
        self.elections_won += 1
        followers = self.ml.alive(include_self=False)
        if getattr(self, "on_round_start", None):
            self.on_round_start()
        reqs = [self.ep.request(f, MsgType.COORDINATE, {"leader": me}, timeout=2 * self.timeout) for f in followers]
        acks: Dict[str, dict] = {}
        for f, r in zip(followers, await asyncio.gather(*reqs)):
            if r is not None:
                acks[f] = r.payload
        log.info("%s elected leader (%d acks)", me, len(acks))
        if self.on_elected:
            self.on_elected(acks)
        if self.on_new_leader:
            self.on_new_leader(me)

    async def _on_election(self, fr: Frame) -> None:
        me = self.ml.self_name
        if self.eligible(me) and self.priority(me) > self.priority(fr.sender):
            await self.ep.send(fr.sender, MsgType.ELECTION_OK, {})
            if self.leader == me:
                await self.ep.send(fr.sender, MsgType.COORDINATE, {"leader": me})
            elif not self.in_election:
                self.trigger()

    async def _on_ok(self, fr: Frame) -> None:
        self._ok.set()

    async def _on_coordinate(self, fr: Frame) -> None:
        new = fr.payload.get("leader", fr.sender)
        self.leader = new
        self._coord.set()
        if fr.seq:
            await self.ep.reply(fr, MsgType.COORDINATE_ACK, self.ack_payload())
        if self.on_new_leader:
            self.on_new_leader(new)

    def set_leader(self, name: Optional[str]) -> None:
        self.leader = name
