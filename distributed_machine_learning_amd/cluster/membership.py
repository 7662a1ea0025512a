"""SWIM-style membership list (pure state machine, injectable clock).

Reference (membershipList.py:14-154): dict "host:port" -> (timestamp, status),
last-writer-wins on timestamps from different hosts' clocks, suspicion = status
0, removal after CLEANUP_TIME, ring of [i+1, i-1, i+4] over a static 10-node
table with substitutes (membershipList.py:61-95, config.py:67-89).

Here: SWIM semantics — every member has an ``incarnation`` that
only its owner increments; state precedence ALIVE < SUSPECT < DEAD for equal
incarnations; a node that hears itself suspected refutes by bumping its
incarnation (so clock skew never decides liveness). Suspects are confirmed DEAD
after ``suspect_timeout`` and purged after ``cleanup_time``; callbacks fire on
join / failure (leader failure -> election, worker failure -> requeue its batch,
any failure -> re-replicate its files; membershipList.py:39-52). The probe ring
is the reference's [+1, -1, +4] offsets over the sorted alive members.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from enum import IntEnum
from typing import Callable, Dict, Iterable, List, Optional, Sequence


class Status(IntEnum):
    ALIVE = 1
    SUSPECT = 2
    DEAD = 3
    LEFT = 4


_PRECEDENCE = {Status.ALIVE: 0, Status.SUSPECT: 1, Status.DEAD: 2, Status.LEFT: 2}


@dataclass
class Member:
    name: str
    incarnation: int
    status: Status
    since: float                      # local time of the last status change
    meta: Dict = field(default_factory=dict)  # role, rank, gpu, ...


Callback = Callable[[str], None]


class MembershipList:
    def __init__(self, self_name: str, clock: Callable[[], float] = time.monotonic, suspect_timeout: float = 3.0,
                 cleanup_time: float = 10.0, meta: Optional[Dict] = None, ring_offsets: Sequence[int] = (1, -1, 4),
                 incarnation: Optional[int] = None):
        self.self_name = self_name
        self.clock = clock
        self.suspect_timeout = suspect_timeout
        self.cleanup_time = cleanup_time
        self.ring_offsets = tuple(ring_offsets)
        inc = incarnation if incarnation is not None else int(time.time() * 1000)
        self.members: Dict[str, Member] = {self_name: Member(self_name, inc, Status.ALIVE, clock(), dict(meta or {}))}
        self.on_join: List[Callback] = []
        self.on_fail: List[Callback] = []      # confirmed dead (or left)
        self.on_suspect: List[Callback] = []
        self.on_purge: List[Callback] = []
        # detector quality counters (reference menu option 10: false-positive rate)
        self.suspicions = 0
        self.false_positives = 0
        self.failures = 0
        self.removed_count = 0
        self._suspected_by_me: set = set()

    # ------------------------------------------------------------ queries --
    @property
    def me(self) -> Member:
        return self.members[self.self_name]

    def get(self, name: str) -> Optional[Member]:
        return self.members.get(name)

    def is_alive(self, name: str) -> bool:
        m = self.members.get(name)
        return m is not None and m.status in (Status.ALIVE, Status.SUSPECT)

    def alive(self, include_self: bool = True, role: Optional[str] = None) -> List[str]:
        out = [n for n, m in self.members.items() if m.status in (Status.ALIVE, Status.SUSPECT)
               and (include_self or n != self.self_name) and (role is None or m.meta.get("role") == role)]
        return sorted(out)

    def ring_targets(self) -> List[str]:
        """Probe targets: [+1, -1, +4] neighbours of self over the sorted alive ring."""
        ring = self.alive(include_self=True)
        if len(ring) <= 1 or self.self_name not in ring:  # self LEFT / not alive: nothing to probe
            return []
        i = ring.index(self.self_name)
        out: List[str] = []
        for off in self.ring_offsets:
            t = ring[(i + off) % len(ring)]
            if t != self.self_name and t not in out:
                out.append(t)
        return out

    def digest(self) -> Dict[str, list]:
        """Gossip payload: every known member (clusters here are <= tens of nodes)."""
        return {n: [m.incarnation, int(m.status), m.meta] for n, m in self.members.items()}

    # ---------------------------------------------------------- mutations --
    def merge(self, digest: Dict[str, list]) -> None:
        for name, entry in digest.items():
            inc, st = int(entry[0]), Status(int(entry[1]))
            meta = entry[2] if len(entry) > 2 and isinstance(entry[2], dict) else {}
            self._apply(name, inc, st, meta)

    def _apply(self, name: str, inc: int, st: Status, meta: Dict) -> None:
        now = self.clock()
        if name == self.self_name:
            me = self.me
            if st in (Status.SUSPECT, Status.DEAD) and inc >= me.incarnation:
                me.incarnation = inc + 1  # refute
                me.since = now
            return
        cur = self.members.get(name)
        if cur is None:
            self.members[name] = Member(name, inc, st, now, dict(meta))
            if st in (Status.ALIVE, Status.SUSPECT):
                self._fire(self.on_join, name)
            elif st in (Status.DEAD, Status.LEFT):
                self.failures += 0  # tombstone of a node we never saw alive: no callback
            return
        newer = inc > cur.incarnation or (inc == cur.incarnation and _PRECEDENCE[st] > _PRECEDENCE[cur.status])
        if not newer:
            return
        old = cur.status
        if meta:
            cur.meta.update(meta)
        cur.incarnation = inc
        if st == old:
            return
        if old in (Status.DEAD, Status.LEFT) and st in (Status.ALIVE, Status.SUSPECT):
            # rejoin with a higher incarnation
            cur.status, cur.since = st, now
            self._fire(self.on_join, name)
            return
        if old == Status.SUSPECT and st == Status.ALIVE and name in self._suspected_by_me:
            self.false_positives += 1
            self._suspected_by_me.discard(name)
        cur.status, cur.since = st, now
        if st == Status.SUSPECT:
            self._fire(self.on_suspect, name)
        elif st in (Status.DEAD, Status.LEFT) and old in (Status.ALIVE, Status.SUSPECT):
            self.failures += 1
            self._fire(self.on_fail, name)

    def suspect(self, name: str) -> None:
        m = self.members.get(name)
        if m is None or name == self.self_name or m.status != Status.ALIVE:
            return
        self.suspicions += 1
        self._suspected_by_me.add(name)
        m.status, m.since = Status.SUSPECT, self.clock()
        self._fire(self.on_suspect, name)

    def mark_alive(self, name: str, inc: Optional[int] = None) -> None:
        """Direct evidence (ACK) that `name` is alive."""
        m = self.members.get(name)
        if m is None:
            return
        if m.status == Status.SUSPECT and (inc is None or inc >= m.incarnation):
            # our own suspicion was wrong
            if name in self._suspected_by_me:
                self.false_positives += 1
                self._suspected_by_me.discard(name)
            m.status, m.since = Status.ALIVE, self.clock()
        if inc is not None and inc > m.incarnation:
            m.incarnation = inc

    def leave(self) -> None:
        self.me.status = Status.LEFT
        self.me.incarnation += 1

    def tick(self) -> None:
        """Advance timers: SUSPECT -> DEAD after suspect_timeout, purge after cleanup_time."""
        now = self.clock()
        for name, m in list(self.members.items()):
            if name == self.self_name:
                continue
            if m.status == Status.SUSPECT and now - m.since >= self.suspect_timeout:
                m.status, m.since = Status.DEAD, now
                self._suspected_by_me.discard(name)
                self.failures += 1
                self._fire(self.on_fail, name)
            elif m.status in (Status.DEAD, Status.LEFT) and now - m.since >= self.cleanup_time:
                del self.members[name]
                self.removed_count += 1
                self._fire(self.on_purge, name)

    def false_positive_rate(self) -> float:
        return self.false_positives / self.suspicions if self.suspicions else 0.0

    def _fire(self, cbs: Iterable[Callback], name: str) -> None:
        for cb in list(cbs):
            cb(name)

    def table(self) -> List[Dict]:
        """For the CLI (reference menu option 1, membershipList.py:141-154)."""
        return [{"node": n, "incarnation": m.incarnation, "status": m.status.name, **m.meta}
                for n, m in sorted(self.members.items())]
