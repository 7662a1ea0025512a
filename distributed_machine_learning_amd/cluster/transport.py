"""Control-plane transports and the request/response endpoint.

* ``UdpTransport`` — asyncio datagram endpoint (reference transport.py:8-34,
  protocol.py:13-81). Differences: frames are MTU-sized fragments (frames.py);
  received datagrams go straight into an asyncio.Queue (the reference's
  Condition+deque ``recv`` waits even when the queue is non-empty, so a backlog
  never drains); test mode drops a deterministic fraction of sends (reference:
  3 %, protocol.py:10) and counts bytes for the bytes/s meter (menu option 9).
* ``LoopbackNetwork`` / ``LoopbackTransport`` — in-process network for tests:
  injectable drop rate, partitions, killed nodes, latency.
* ``Endpoint`` — handler dispatch plus per-request futures keyed by ``seq``
  (replaces the single ``_waiting_for_leader_event`` slot that let concurrent
  client operations race, worker.py:1123-1135).
"""
from __future__ import annotations

import asyncio
import itertools
import logging
import random
import time
from typing import Awaitable, Callable, Dict, Optional, Set, Tuple

from .frames import Frame, FrameError, MsgType, Reassembler, encode
from .tasks import spawn

log = logging.getLogger(__name__)
Addr = Tuple[str, int]


def addr_of(name: str) -> Addr:
    host, port = name.rsplit(":", 1)
    return host, int(port)


def name_of(addr: Addr) -> str:
    return f"{addr[0]}:{addr[1]}"


class Transport:
    """Abstract datagram transport carrying whole Frames."""

    name: str
    bytes_sent: int = 0
    bytes_recv: int = 0
    drop_rate: float = 0.0

    async def send(self, dest: str, frame: Frame) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    async def recv(self) -> Frame:  # pragma: no cover - interface
        raise NotImplementedError

    def close(self) -> None:  # pragma: no cover - interface
        pass


class _DropPolicy:
    """Deterministic pseudo-random drop (seeded) so test runs are reproducible."""

    def __init__(self, rate: float, seed: int):
        self.rate = rate
        self.rng = random.Random(seed)

    def drop(self) -> bool:
        return self.rate > 0 and self.rng.random() < self.rate


class UdpTransport(Transport):
    def __init__(self, host: str, port: int, drop_rate: float = 0.0, seed: int = 0):
        self.host, self.port = host, port
        self.name = f"{host}:{port}"
        self.drop_rate = drop_rate
        self._drop = _DropPolicy(drop_rate, seed ^ port)
        self._q: asyncio.Queue = asyncio.Queue()
        self._reasm = Reassembler()
        self._tr: Optional[asyncio.DatagramTransport] = None
        self.bytes_sent = 0
        self.bytes_recv = 0
        self.started = time.monotonic()

    async def start(self) -> "UdpTransport":
        loop = asyncio.get_running_loop()
        outer = self

        class _P(asyncio.DatagramProtocol):
            def datagram_received(self, data, addr):
                outer.bytes_recv += len(data)
                try:
                    fr = outer._reasm.feed(data)
                except FrameError as e:
                    log.debug("dropping bad datagram from %s: %s", addr, e)
                    return
                if fr is not None:
                    outer._q.put_nowait(fr)

        self._tr, _ = await loop.create_datagram_endpoint(_P, local_addr=(self.host, self.port))
        if self.port == 0:
            self.port = self._tr.get_extra_info("sockname")[1]
            self.name = f"{self.host}:{self.port}"
        return self

    async def send(self, dest: str, frame: Frame) -> None:
        if self._tr is None:
            raise RuntimeError("transport not started")
        if dest == self.name:  # to this node itself (e.g. the store leader is one of the replicas): no socket
            self._q.put_nowait(frame)
            return
        if self._drop.drop():
            return
        addr = addr_of(dest)
        for dg in encode(frame):
            self.bytes_sent += len(dg)
            self._tr.sendto(dg, addr)

    async def recv(self) -> Frame:
        return await self._q.get()

    def bps(self) -> float:
        return self.bytes_sent / max(1e-9, time.monotonic() - self.started)

    def close(self) -> None:
        if self._tr is not None:
            self._tr.close()
            self._tr = None


class LoopbackNetwork:
    """In-memory network: name -> queue, with drop / partition / kill / latency injection."""

    def __init__(self, drop_rate: float = 0.0, seed: int = 0, latency: float = 0.0):
        self.nodes: Dict[str, "LoopbackTransport"] = {}
        self.drop = _DropPolicy(drop_rate, seed)
        self.latency = latency
        self.blocked: Set[Tuple[str, str]] = set()
        self.dead: Set[str] = set()
        self.delivered = 0

    def transport(self, name: str) -> "LoopbackTransport":
        t = LoopbackTransport(self, name)
        self.nodes[name] = t
        return t

    def partition(self, a: str, b: str) -> None:
        self.blocked |= {(a, b), (b, a)}

    def heal(self) -> None:
        self.blocked.clear()

    def kill(self, name: str) -> None:
        self.dead.add(name)

    def revive(self, name: str) -> None:
        self.dead.discard(name)

    def set_drop_rate(self, rate: float) -> None:
        self.drop.rate = rate

    async def deliver(self, src: str, dest: str, frame: Frame) -> None:
        if src in self.dead or dest in self.dead or (src, dest) in self.blocked or self.drop.drop():
            return
        t = self.nodes.get(dest)
        if t is None:
            return
        # round-trip through the codec so tests exercise the real wire format
        from .frames import Reassembler

        r = Reassembler()
        out = None
        for dg in encode(frame):
            t.bytes_recv += len(dg)
            out = r.feed(dg)
        if self.latency:
            await asyncio.sleep(self.latency)
        self.delivered += 1
        t._q.put_nowait(out)


class LoopbackTransport(Transport):
    def __init__(self, net: LoopbackNetwork, name: str):
        self.net, self.name = net, name
        self._q: asyncio.Queue = asyncio.Queue()
        self.bytes_sent = 0
        self.bytes_recv = 0

    async def send(self, dest: str, frame: Frame) -> None:
        self.bytes_sent += sum(len(d) for d in encode(frame))
        if self.net.latency:
            spawn(self.net.deliver(self.name, dest, frame))
        else:
            await self.net.deliver(self.name, dest, frame)

    async def recv(self) -> Frame:
        return await self._q.get()


Handler = Callable[[Frame], Awaitable[None]]


class Endpoint:
    """Dispatches incoming frames to handlers; matches replies to pending requests."""

    _seq = itertools.count(1)

    def __init__(self, transport: Transport):
        self.t = transport
        self.name = transport.name
        self.handlers: Dict[MsgType, Handler] = {}
        self.pending: Dict[int, asyncio.Future] = {}
        self._task: Optional[asyncio.Task] = None
        self.default_handler: Optional[Handler] = None
        self.stopped = False

    def on(self, mtype: MsgType, handler: Handler) -> None:
        self.handlers[mtype] = handler

    def start(self) -> asyncio.Task:
        self._task = asyncio.get_running_loop().create_task(self._run())
        return self._task

    async def _run(self) -> None:
        while not self.stopped:
            fr = await self.t.recv()
            if fr.is_reply and fr.seq in self.pending:
                fut = self.pending.pop(fr.seq)
                if not fut.done():
                    fut.set_result(fr)
                continue
            h = self.handlers.get(fr.type, self.default_handler)
            if h is None:
                log.debug("%s: no handler for %s", self.name, fr.type.name)
                continue
            spawn(self._safe(h, fr))

    async def _safe(self, h: Handler, fr: Frame) -> None:
        try:
            await h(fr)
        except Exception:  # handler bugs must not kill the dispatch loop
            log.exception("%s: handler for %s failed", self.name, fr.type.name)

    async def send(self, dest: str, mtype: MsgType, payload: Optional[dict] = None, seq: int = 0,
                   reply: bool = False) -> None:
        await self.t.send(dest, Frame(mtype, self.name, payload or {}, seq, 1 if reply else 0))

    async def reply(self, req: Frame, mtype: MsgType, payload: Optional[dict] = None) -> None:
        await self.send(req.sender, mtype, payload, seq=req.seq, reply=True)

    async def request(self, dest: str, mtype: MsgType, payload: Optional[dict] = None, timeout: float = 2.0,
                      retries: int = 0) -> Optional[Frame]:
        """Send and await the reply with the same seq (None on timeout after retries)."""
        for _ in range(retries + 1):
            seq = next(self._seq)
            fut = asyncio.get_running_loop().create_future()
            self.pending[seq] = fut
            await self.send(dest, mtype, payload, seq=seq)
            try:
                return await asyncio.wait_for(fut, timeout)
            except asyncio.TimeoutError:
                pass
            finally:  # timed out, answered or cancelled by the caller: never leave the entry behind
                self.pending.pop(seq, None)
        return None

    def stop(self) -> None:
        self.stopped = True
        if self._task:
            self._task.cancel()
        for f in self.pending.values():
            if not f.done():
                f.cancel()
        self.pending.clear()
        self.t.close()
