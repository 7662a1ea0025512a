"""Bulk-byte data plane between store nodes (replaces asyncssh scp).

Reference: every replica scp-pulls from the client on PUT (file_service.py:
76-77), re-replication scp's a wildcard of every version (:54-55), GET scp's
to a local destination (:119-120) — one SSH connection per image, ~1 s/image
(test.py:109), with a plaintext password in config.

Here every node runs a tiny asyncio TCP blob server next to its control
endpoint; a request is one JSON line, the answer is length-prefixed bytes.
Sources: the node's versioned store, or its short-lived *outbox* (bytes a client
is PUTting, held until every replica has pulled them). ``InProcBlobNetwork``
provides the same interface for in-process tests.
"""
from __future__ import annotations

import asyncio
import logging
import json
import struct
import uuid
from typing import Dict, List, Optional, Tuple

from .local_store import LocalFileStore

_LEN = struct.Struct(">qI")  # length (-1 = not found), version

log = logging.getLogger(__name__)


class BlobSource:
    """What a node serves: its store + an outbox of pending PUT payloads."""

    def __init__(self, store: LocalFileStore):
        self.store = store
        self.outbox: Dict[str, bytes] = {}

    def stage(self, data) -> str:
        """Hold ``data`` (bytes, or {name: bytes} for a multi-file PUT) until unstaged."""
        tok = uuid.uuid4().hex
        self.outbox[tok] = data
        return tok

    def unstage(self, tok: str) -> None:
        self.outbox.pop(tok, None)

    def read(self, req: dict) -> List[Tuple[int, bytes]]:
        op = req.get("op")
        if op == "outbox":
            data = self.outbox.get(req["token"])
            return [] if data is None else [(0, data)]
        if op == "outbox_many":  # the named files of a staged bundle, in request order
            box = self.outbox.get(req["token"])
            if not isinstance(box, dict) or any(n not in box for n in req["names"]):
                return []
            return [(0, box[n]) for n in req["names"]]
        name = req["name"]
        if op == "get":
            v = req.get("version")
            try:
                vv = v if v is not None else self.store.latest(name)
                return [(vv, self.store.get_bytes(name, vv))]
            except (FileNotFoundError, TypeError):
                return []
        if op == "get_all":
            return [(v, self.store.get_bytes(name, v)) for v in self.store.versions(name)]
        return []


class BlobServer:
    def __init__(self, source: BlobSource, host: str = "127.0.0.1", port: int = 0):
        self.source, self.host, self.port = source, host, port
        self._srv: Optional[asyncio.AbstractServer] = None
        self.bytes_served = 0

    async def start(self) -> "BlobServer":
        self._srv = await asyncio.start_server(self._handle, self.host, self.port)
        self.port = self._srv.sockets[0].getsockname()[1]
        return self

    @property
    def addr(self) -> str:
        return f"{self.host}:{self.port}"

    async def _handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        try:
            while True:
                line = await reader.readline()
                if not line:
                    break
                try:
                    items = self.source.read(json.loads(line))
                except (ConnectionError, asyncio.CancelledError):
                    raise
                except Exception as e:  # bad request / name / version evicted mid get_all
                    log.warning("blob server: request failed (%s: %s)", type(e).__name__, e)
                    writer.write(struct.pack(">i", -1))  # explicit error reply, connection stays usable
                    await writer.drain()
                    continue
                writer.write(struct.pack(">i", len(items)))
                for v, data in items:
                    writer.write(_LEN.pack(len(data), v))
                    writer.write(data)
                    self.bytes_served += len(data)
                await writer.drain()
        except (ConnectionError, json.JSONDecodeError):
            pass
        finally:
            writer.close()

    def close(self) -> None:
        if self._srv:
            self._srv.close()


class TcpBlobClient:
    """Fetch from a peer's blob server; the address comes from membership meta."""

    def __init__(self, resolve):
        self.resolve = resolve  # node name -> "host:port" of its blob server
        self.bytes_fetched = 0

    async def fetch(self, node: str, req: dict, timeout: float = 30.0, addr: Optional[str] = None
                    ) -> List[Tuple[int, bytes]]:
        addr = self.resolve(node) or addr
        if addr is None:
            raise ConnectionError(f"no blob address for {node}")
        host, port = addr.rsplit(":", 1)
        reader, writer = await asyncio.wait_for(asyncio.open_connection(host, int(port)), timeout)
        try:
            writer.write((json.dumps(req) + "\n").encode())
            await writer.drain()
            (n,) = struct.unpack(">i", await asyncio.wait_for(reader.readexactly(4), timeout))
            if n < 0:
                raise ConnectionError(f"blob server {node} could not serve {req}")
            out = []
            for _ in range(n):
                ln, v = _LEN.unpack(await asyncio.wait_for(reader.readexactly(_LEN.size), timeout))
                data = await asyncio.wait_for(reader.readexactly(ln), timeout)
                self.bytes_fetched += ln
                out.append((v, data))
            return out
        except asyncio.IncompleteReadError as e:  # peer closed mid-reply: an EOFError, not an OSError
            raise ConnectionError(f"blob server {node} closed the connection mid-reply") from e
        finally:
            writer.close()


class InProcBlobNetwork:
    """Same interface, no sockets (tests): node name -> BlobSource."""

    def __init__(self):
        self.sources: Dict[str, BlobSource] = {}
        self.dead: set = set()

    def register(self, node: str, source: BlobSource) -> None:
        self.sources[node] = source

    async def fetch(self, node: str, req: dict, timeout: float = 30.0, addr: Optional[str] = None
                    ) -> List[Tuple[int, bytes]]:
        if node in self.dead or node not in self.sources:
            raise ConnectionError(node)
        await asyncio.sleep(0)
        return self.sources[node].read(req)
