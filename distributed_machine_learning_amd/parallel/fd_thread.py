"""Host-side SWIM failure detector for the ranks of one collective job.

Each rank runs the cluster/ SWIM detector (UDP on 127.0.0.1:base_port+rank) in
a daemon thread with its own asyncio loop; a rank confirmed dead is added to
``ElasticGroup.dead`` so pending collectives abort and the coordinator starts a
new communicator epoch. This keeps liveness independent of RCCL, which cannot
report a dead peer (SURVEY §2.6 "gossip all-to-all" row).
"""
from __future__ import annotations

import asyncio
import logging
import threading
from typing import Callable, Optional, Set

from ..cluster.failure_detector import FailureDetector
from ..cluster.membership import MembershipList
from ..cluster.transport import Endpoint, UdpTransport
from ..cluster.tasks import spawn

log = logging.getLogger(__name__)


class RankFailureDetector:
    def __init__(self, grank: int, world: int, base_port: int, on_dead: Callable[[int], None],
                 host: str = "127.0.0.1", period: float = 0.1, ping_timeout: float = 0.1,
                 suspect_timeout: float = 0.5, on_alive: Optional[Callable[[int], None]] = None):
        self.grank, self.world, self.base, self.host = grank, world, base_port, host
        self.on_dead, self.on_alive = on_dead, on_alive
        self.period, self.ping_timeout, self.suspect_timeout = period, ping_timeout, suspect_timeout
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.ready = threading.Event()
        self.thread = threading.Thread(target=self._main, daemon=True, name=f"swim-{grank}")
        self.dead: Set[int] = set()

    def name(self, r: int) -> str:
        return f"{self.host}:{self.base + r}"

    def rank_of(self, name: str) -> int:
        return int(name.rsplit(":", 1)[1]) - self.base

    def start(self) -> "RankFailureDetector":
        import atexit

        self.thread.start()
        self.ready.wait(10)
        # a process that leaves without stop() (an exception unwinding the rank)
        # must not tear the daemon thread's loop down with its tasks pending
        atexit.register(self.stop)
        return self

    def _main(self) -> None:
        self.loop = asyncio.new_event_loop()
        asyncio.set_event_loop(self.loop)
        # the loop keeps only a weak reference to a task: without this one, the garbage
        # collector destroys the pending detector task (and with it its objects) mid-run
        self._task = spawn(self._run(), self.loop)
        self.loop.run_forever()
        # drain anything stop() did not reach (e.g. it timed out) before closing
        pending = [t for t in asyncio.all_tasks(self.loop) if not t.done()]
        for t in pending:
            t.cancel()
        if pending:
            self.loop.run_until_complete(asyncio.gather(*pending, return_exceptions=True))
        self.loop.close()

    async def _run(self) -> None:
        t = await UdpTransport(self.host, self.base + self.grank).start()
        ep = Endpoint(t)
        ml = MembershipList(t.name, suspect_timeout=self.suspect_timeout, cleanup_time=30.0,
                            meta={"role": "worker", "rank": self.grank})
        # every rank knows the static job membership up front (torchrun world)
        ml.merge({self.name(r): [0, 1, {"rank": r}] for r in range(self.world) if r != self.grank})

        def failed(name: str) -> None:
            r = self.rank_of(name)
            if r not in self.dead:
                self.dead.add(r)
                log.warning("rank %d: SWIM confirmed rank %d dead", self.grank, r)
                self.on_dead(r)

        def joined(name: str) -> None:  # a dead rank's restarted process (higher incarnation)
            r = self.rank_of(name)
            if r in self.dead:
                self.dead.discard(r)
                log.warning("rank %d: SWIM saw rank %d rejoin", self.grank, r)
                if self.on_alive is not None:
                    self.on_alive(r)

        ml.on_fail.append(failed)
        ml.on_join.append(joined)
        self.fd = FailureDetector(ep, ml, period=self.period, ping_timeout=self.ping_timeout)
        ep.start()
        self.fd.start()
        self.ready.set()
        self._idle = asyncio.Event()  # held by self: the parked task stays reachable
        await self._idle.wait()

    async def _shutdown(self) -> None:
        for stop in (getattr(self.fd, "stop", None), getattr(getattr(self.fd, "ep", None), "stop", None)):
            try:
                if stop is not None:
                    stop()
            except Exception:  # pragma: no cover - best effort at exit
                pass
        tasks = [t for t in asyncio.all_tasks() if t is not asyncio.current_task()]
        for t in tasks:
            t.cancel()
        await asyncio.gather(*tasks, return_exceptions=True)

    def stop(self) -> None:
        """Cancel the detector's tasks, close its socket and join the thread."""
        if self.loop is None or not self.thread.is_alive():
            return
        try:
            asyncio.run_coroutine_threadsafe(self._shutdown(), self.loop).result(timeout=5)
        except Exception:  # pragma: no cover - best effort at exit
            pass
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.thread.join(timeout=5)
