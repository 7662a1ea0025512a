"""Worker role: execute one batch per WORKER_TASK_REQUEST.

Reference (worker.py:518-537, 940-962, 1361-1386, 1573-1585): on a task the
worker cancels whatever it was running, scp-downloads each image SEQUENTIALLY
(~1 s/image), runs the batch in a fresh process that rebuilds the model, dumps
``output_<job>_<batch>_<host>.json``, PUTs it into SDFS and ACKs the leader with
``{jobid, batchid, model, image_count, start_time}`` (start_time on the worker's
clock).

Here: images are read from the local replica or fetched from holders
CONCURRENTLY over the blob plane; decoding runs on a thread pool; the model is
resident in the backend (HBM for the GPU backend); the ACK carries the
worker-measured service time and is retried until the coordinator confirms.
"""
from __future__ import annotations

import asyncio
import logging
import os
import time
from typing import Callable, Dict, List, Optional

from ..cluster.frames import Frame, MsgType
from ..cluster.transport import Endpoint
from ..store.service import StoreService
from .inference import Backend
from .output import decode_top5, dumps, output_name

log = logging.getLogger(__name__)


class WorkerRole:
    def __init__(self, ep: Endpoint, store: StoreService, backend: Backend,
                 coordinator_fn: Callable[[], Optional[str]], host_tag: str, out_dir: Optional[str] = None,
                 fetch_concurrency: int = 16):
        self.ep, self.store, self.backend = ep, store, backend
        self.coordinator_fn = coordinator_fn
        self.host_tag = host_tag
        self.out_dir = out_dir
        self.sem = asyncio.Semaphore(fetch_concurrency)
        self.current: Optional[asyncio.Task] = None
        self.current_key = None
        self.completed = 0
        self.cancelled = 0
        self.enabled = True
        ep.on(MsgType.WORKER_TASK_REQUEST, self._on_task)
        ep.on(MsgType.WORKER_KILL_TASK_REQUEST, self._on_kill)

    async def _on_task(self, fr: Frame) -> None:
        if not self.enabled:
            return
        await self.ep.reply(fr, MsgType.ACK, {"accepted": True})
        await self._cancel_current()
        self.current_key = (fr.payload["jobid"], fr.payload["batchid"])
        self.current = asyncio.get_running_loop().create_task(self.run_task(fr.payload, fr.sender))

    async def _on_kill(self, fr: Frame) -> None:
        await self._cancel_current()
        await self.ep.reply(fr, MsgType.WORKER_KILL_TASK_REQUEST_ACK, {"jobid": fr.payload.get("jobid")})

    async def _cancel_current(self) -> None:
        if self.current is not None and not self.current.done():
            self.current.cancel()
            self.cancelled += 1
            try:
                await self.current
            except (asyncio.CancelledError, Exception):
                pass

    async def _fetch(self, name: str, holders: Dict[str, List[int]]) -> Optional[bytes]:
        async with self.sem:
            if self.store.local.has(name):
                return self.store.local.get_bytes(name)
            got = await self.store.fetch_from(holders, name)
            return None if got is None else got[1]

    async def run_task(self, p: dict, coordinator: str) -> dict:
        t0 = time.monotonic()
        job, batch, model = int(p["jobid"]), int(p["batchid"]), p["model"]
        images: Dict[str, Dict[str, List[int]]] = p["images"]
        names = list(images)
        blobs = await asyncio.gather(*(self._fetch(n, images[n]) for n in names))
        ok = [(n, b) for n, b in zip(names, blobs) if b is not None]
        failed = [n for n, b in zip(names, blobs) if b is None]
        loop = asyncio.get_running_loop()
        result: Dict[str, object] = {}
        if ok:
            arr = await loop.run_in_executor(None, self.backend.decode_batch, model, [b for _, b in ok])
            idx, prob = await loop.run_in_executor(None, self.backend.predict, model, arr)
            result = decode_top5([n for n, _ in ok], idx, prob, failed)
        else:
            result = decode_top5([], [], [], failed)
        service = time.monotonic() - t0
        fname = output_name(job, batch, self.host_tag)
        text = dumps(result)
        if self.out_dir:
            os.makedirs(self.out_dir, exist_ok=True)
            with open(os.path.join(self.out_dir, fname), "w") as f:
                f.write(text)
        await self.store.put(text.encode(), fname)
        ack = {"jobid": job, "batchid": batch, "model": model, "image_count": len(names),
               "service_time": service, "start_time": time.time() - service, "output": fname}
        for _ in range(10):
            dest = self.coordinator_fn()
            if dest is None:
                await asyncio.sleep(0.2)
                continue
            r = await self.ep.request(dest, MsgType.WORKER_TASK_REQUEST_ACK, ack, timeout=1.0)
            if r is not None:
                break
        self.completed += 1
        self.current_key = None
        return ack
