"""Introducer "DNS": a tiny service that names the current leader.

Reference: a separate UDP process on port 8888 (``introduce process/``;
handler worker.py:43-62 there). FETCH_INTRODUCER returns the current
introducer/leader ``host:port``; UPDATE_INTRODUCER sets it to the sender. It
defaults to H1 (introduce process/config.py:96).
"""
from __future__ import annotations

import asyncio
import logging
from typing import Optional

from .frames import Frame, MsgType
from .transport import Endpoint, UdpTransport

log = logging.getLogger(__name__)


class IntroducerService:
    def __init__(self, ep: Endpoint, default_leader: Optional[str] = None):
        self.ep = ep
        self.leader = default_leader
        self.updates = 0
        ep.on(MsgType.FETCH_INTRODUCER, self._on_fetch)
        ep.on(MsgType.UPDATE_INTRODUCER, self._on_update)

    async def _on_fetch(self, fr: Frame) -> None:
        if self.leader is None:  # first node to ask becomes the introducer
            self.leader = fr.sender
        await self.ep.reply(fr, MsgType.FETCH_INTRODUCER_ACK, {"introducer": self.leader})

    async def _on_update(self, fr: Frame) -> None:
        self.leader = fr.payload.get("leader", fr.sender)
        self.updates += 1
        log.info("introducer now %s", self.leader)
        await self.ep.reply(fr, MsgType.FETCH_INTRODUCER_ACK, {"introducer": self.leader})


async def fetch_leader(ep: Endpoint, dns: str, timeout: float = 1.0, retries: int = 3) -> Optional[str]:
    r = await ep.request(dns, MsgType.FETCH_INTRODUCER, {}, timeout=timeout, retries=retries)
    return None if r is None else r.payload.get("introducer")


async def update_leader(ep: Endpoint, dns: str, leader: str, timeout: float = 1.0) -> bool:
    r = await ep.request(dns, MsgType.UPDATE_INTRODUCER, {"leader": leader}, timeout=timeout, retries=2)
    return r is not None


async def serve(host: str, port: int, default_leader: Optional[str] = None) -> None:
    """Run the introducer as its own process (``python -m ...cluster.introducer``)."""
    t = await UdpTransport(host, port).start()
    ep = Endpoint(t)
    IntroducerService(ep, default_leader)
    ep.start()
    log.info("introducer listening on %s", t.name)
    await asyncio.Event().wait()


if __name__ == "__main__":  # pragma: no cover
    import argparse

    ap = argparse.ArgumentParser(description="introducer DNS (reference: introduce process/main.py)")
    ap.add_argument("-H", "--hostname", default="127.0.0.1")
    ap.add_argument("-p", "--port", type=int, default=8888)
    ap.add_argument("--leader", default=None)
    a = ap.parse_args()
    logging.basicConfig(level=logging.INFO)
    asyncio.run(serve(a.hostname, a.port, a.leader))
