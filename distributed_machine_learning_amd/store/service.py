"""The replicated, versioned store ("SDFS") protocol: leader, replica, client.

Reference protocol (worker.py:651-883 handlers, 1201-1354 client, leader.py):
PUT -> leader picks 4 replicas, each scp-pulls from the client, leader reports
success when all did; GET asks the leader for holders then pulls from the first
that works (R = 1); DELETE fans out; LS / LS-ALL / GET-VERSIONS are leader
queries; after failures the leader re-replicates under-replicated files.

Same semantics here, over request/reply frames (per-request futures) and the
blob data plane (store/blob.py). Fixed reference defects: failed PUTs are
reported (leader.py:132 typo), a dead replica of an in-flight PUT is replaced
(worker.py:1264 inverted test), placement never loops forever (leader.py:60),
``put`` never waits without a timeout (worker.py:1546).
"""
from __future__ import annotations

import asyncio
import logging
import os
import shutil
import socket
import time
import uuid
from typing import Callable, Dict, List, Optional, Tuple

from ..cluster.frames import Frame, MsgType
from ..cluster.membership import MembershipList
from ..cluster.transport import Endpoint
from .blob import BlobSource
from .local_store import LocalFileStore
from .metadata import FAILED, SUCCESS, StoreMetadata

log = logging.getLogger(__name__)


def _host_id() -> str:
    """This machine's identity for the same-node fast path (hostname + kernel boot id):
    a spool path is only ever linked by a replica that sees the same filesystem."""
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        boot = ""
    return f"{socket.gethostname()}/{boot}"


HOST_ID = _host_id()


class StoreService:
    def __init__(self, ep: Endpoint, ml: MembershipList, local: LocalFileStore, source: BlobSource, blobs,
                 leader_fn: Callable[[], Optional[str]], replication: int = 4, timeout: float = 10.0,
                 storage_role: Optional[Callable[[str], bool]] = None):
        self.ep, self.ml, self.local, self.source, self.blobs = ep, ml, local, source, blobs
        self.leader_fn = leader_fn
        self.meta = StoreMetadata(replication)
        self.timeout = timeout
        self.storage_role = storage_role or (lambda n: True)
        # same-node bundle PUTs (put_many with a spool): the client writes each file once
        # into spool_root/<token>/, every replica on this machine hard-links it into its own
        # versioned store; replicas elsewhere pull it over the blob plane as before
        self.spool_root = os.path.join(os.path.dirname(os.path.abspath(local.root)), ".spool")
        self.linked = 0
        self.pulled = 0
        # leader-side: set while the file map is settled; cleared from the start of a COORDINATE
        # round until adopt() (a listing answered in between came from a half-built map)
        self._settled = asyncio.Event()
        self._settled.set()
        # client-side listings (ls / ls-all: get-output) wait this long for a reachable, settled
        # leader across an election instead of answering "nothing" (reference: the client
        # blocks on the leader, worker.py:1123-1135)
        self.query_wait_s = 20.0
        on = ep.on
        # leader-side
        on(MsgType.PUT_REQUEST, self._l_put)
        on(MsgType.PUT_MANY_REQUEST, self._l_put_many)
        on(MsgType.DELETE_FILE_REQUEST, self._l_delete)
        on(MsgType.LIST_FILE_REQUEST, self._l_ls)
        on(MsgType.GET_FILE_REQUEST, self._l_get)
        on(MsgType.GET_FILE_NAMES_REQUEST, self._l_ls_all)
        on(MsgType.ALL_LOCAL_FILES, self._l_all_local_files)
        on(MsgType.FILES_STORED, self._l_files_stored)
        # replica-side
        on(MsgType.DOWNLOAD_FILE, self._r_download)
        on(MsgType.DOWNLOAD_MANY, self._r_download_many)
        on(MsgType.DELETE_FILE, self._r_delete)
        on(MsgType.REPLICATE_FILE, self._r_replicate)

    # ------------------------------------------------------------ helpers --
    _round: Optional[Dict[str, Dict[str, list]]] = None  # node -> files reported during a COORDINATE round

    @property
    def me(self) -> str:
        return self.ep.name

    def is_leader(self) -> bool:
        return self.leader_fn() == self.me

    def storage_nodes(self) -> List[str]:
        return [n for n in self.ml.alive() if self.storage_role(n)]

    async def _leader_request(self, mtype: MsgType, payload: dict, timeout: Optional[float] = None) -> Optional[Frame]:
        leader = self.leader_fn()
        if leader is None:
            return None
        return await self.ep.request(leader, mtype, payload, timeout=timeout or self.timeout, retries=1)

    # ========================================================== client API ==
    async def put(self, data: bytes, name: str) -> Tuple[bool, str]:
        tok = self.source.stage(data)
        me = self.ml.get(self.me)
        # our blob address rides along: replicas may not have our membership
        # metadata yet right after we joined
        blob = me.meta.get("blob") if me is not None else None
        try:
            r = await self._leader_request(MsgType.PUT_REQUEST, {"filename": name, "token": tok, "blob": blob},
                                           timeout=self.timeout * 3)
        finally:
            self.source.unstage(tok)
        if r is None:
            return False, "leader unreachable"
        return r.type == MsgType.PUT_REQUEST_SUCCESS, r.payload.get("error", "")

    def spool(self, items: List[Tuple[str, bytes]]) -> str:
        """(any thread) Write a bundle's files once into a fresh spool directory on this
        machine's filesystem; put_many(spool=...) then lets same-node replicas hard-link
        them instead of pulling the bytes over TCP. Returns the directory."""
        from .fastio import spool_write

        os.makedirs(self.spool_root, exist_ok=True)
        d = os.path.join(self.spool_root, uuid.uuid4().hex)
        spool_write(d, items)   # one native call for the bundle (GIL released once)
        return d

    async def put_many(self, items: List[Tuple[str, bytes]], spool: Optional[str] = None
                       ) -> Tuple[List[str], List[str], str]:
        """PUT several files in ONE leader round trip (the service's output bundles):
        the leader sends each replica one DOWNLOAD_MANY for all its files of the
        bundle, which it pulls in one blob request — or, when the bundle was spooled on
        this machine (``spool``, from :meth:`spool`) and the replica runs here too, links
        from the spool. Returns (stored, failed, error); every file is stored on all of
        its replicas or reported failed (W = all)."""
        box = dict(items)
        tok = self.source.stage(box)
        me = self.ml.get(self.me)
        blob = me.meta.get("blob") if me is not None else None
        req = {"files": list(box), "token": tok, "blob": blob}
        if spool is not None:
            req.update(spool=spool, host=HOST_ID)
        try:
            r = await self._leader_request(MsgType.PUT_MANY_REQUEST, req, timeout=self.timeout * 3)
        finally:
            self.source.unstage(tok)
        if r is None:
            return [], list(box), "leader unreachable"
        return list(r.payload.get("ok", [])), list(r.payload.get("failed", [])), r.payload.get("error", "")

    async def put_many_direct(self, items: List[Tuple[str, bytes]], spool: Optional[str] = None
                              ) -> Tuple[List[str], List[str], str]:
        """Leaderless bundle PUT for files whose names no other writer uses at the same time
        (the collective service's outputs: one name per (job, batch), r5). The writer places
        each file itself (the same deterministic ring as the leader, over its own view of the
        alive storage nodes), sends each replica node one DOWNLOAD_MANY for all of its files
        (hard links from the spool on this machine, else one blob pull), substitutes a replica
        that dies mid-PUT, and tells the leader what landed where in ONE FILES_STORED message.
        The leader's event loop, which serves every rank's bundles, then handles one small
        message per bundle instead of a fan-out (measured at world 8: PUT p50 133 ms through
        the leader). Versions are assigned by each replica (the next one it holds: a re-run
        of a batch becomes a new version). W = all: a file is stored once every one of its
        targets stored it. Returns (stored, failed, error)."""
        box = dict(items)
        alive = self.storage_nodes()
        if not alive:
            return [], list(box), "no storage nodes"
        tok = self.source.stage(box)
        me = self.ml.get(self.me)
        src = {"source": self.me, "token": tok, "source_blob": me.meta.get("blob") if me is not None else None}
        if spool is not None:
            src.update(spool=spool, host=HOST_ID)
        stored_on: Dict[str, Dict[str, List[int]]] = {n: {} for n in box}
        tried: Dict[str, set] = {}
        pending: Dict[str, List[str]] = {}
        for n in box:
            t = self.meta.place(n, alive)
            tried[n] = set(t)
            for x in t:
                pending.setdefault(x, []).append(n)
        bad: set = set()
        try:
            while pending:
                nodes = sorted(pending)
                rs = await asyncio.gather(*(self._request_unless_dead(
                    t, MsgType.DOWNLOAD_MANY, {"files": [[n, 0] for n in pending[t]], **src}) for t in nodes))
                nxt: Dict[str, List[str]] = {}
                for t, r in zip(nodes, rs):
                    got = r.payload.get("ok", {}) if r is not None else {}
                    dead = r is None and not self.ml.is_alive(t)
                    for n in pending[t]:
                        if n in got:
                            stored_on[n][t] = list(got[n])
                            continue
                        subs = [x for x in self.meta.place(n, self.storage_nodes(), 64) if x not in tried[n]] \
                            if dead else []
                        if subs:  # the replica died mid-PUT: another node takes this file
                            tried[n].add(subs[0])
                            nxt.setdefault(subs[0], []).append(n)
                        else:
                            bad.add(n)
                pending = nxt
        finally:
            self.source.unstage(tok)
        ok = [n for n in box if n not in bad and stored_on[n]]
        failed = [n for n in box if n not in ok]
        if ok:
            per_node: Dict[str, Dict[str, List[int]]] = {}
            for n in ok:
                for node, vers in stored_on[n].items():
                    per_node.setdefault(node, {})[n] = vers
            await self._leader_request(MsgType.FILES_STORED, {"files": per_node})  # None: a new leader adopts
        return ok, failed, "" if not failed else "replica failed"

    async def put_file(self, path: str, name: str) -> Tuple[bool, str]:
        with open(path, "rb") as f:
            return await self.put(f.read(), name)

    async def locate(self, name: str) -> Dict[str, List[int]]:
        r = await self._leader_request(MsgType.GET_FILE_REQUEST, {"filename": name})
        return {} if r is None else r.payload.get("machineids_with_file_versions", {})

    async def get(self, name: str, version: Optional[int] = None) -> Optional[Tuple[int, bytes]]:
        if self.local.has(name, version):
            v = version if version is not None else self.local.latest(name)
            return v, self.local.get_bytes(name, v)
        holders = await self.locate(name)
        return await self.fetch_from(holders, name, version)

    async def fetch_from(self, holders: Dict[str, List[int]], name: str, version: Optional[int] = None
                         ) -> Optional[Tuple[int, bytes]]:
        """R = 1: first holder that answers (the local replica first)."""
        order = sorted(holders, key=lambda n: (n != self.me, n))
        for node in order:
            if version is not None and version not in holders[node]:
                continue
            try:
                items = await self.blobs.fetch(node, {"op": "get", "name": name, "version": version})
            except (ConnectionError, OSError, asyncio.TimeoutError):
                continue
            if items:
                return items[0]
        return None

    async def delete(self, name: str) -> Tuple[bool, str]:
        r = await self._leader_request(MsgType.DELETE_FILE_REQUEST, {"filename": name})
        if r is None:
            return False, "leader unreachable"
        return r.type == MsgType.DELETE_FILE_REQUEST_SUCCESS, r.payload.get("error", "")

    async def _leader_query(self, mtype: MsgType, payload: dict) -> Optional[Frame]:
        """A read-only leader request retried until ``query_wait_s``: right after the leader
        died there is no leader, or a dead one, until SWIM confirms it and the election ends
        (tests/test_elastic_service.py: the coordinator-kill listing raced that election)."""
        t_end = time.monotonic() + self.query_wait_s
        while True:
            r = await self._leader_request(mtype, payload)
            if r is not None or time.monotonic() >= t_end:
                return r
            await asyncio.sleep(0.1)

    async def ls(self, name: str) -> List[str]:
        r = await self._leader_query(MsgType.LIST_FILE_REQUEST, {"filename": name})
        return [] if r is None else r.payload.get("machines", [])

    async def ls_all(self, pattern: str) -> List[str]:
        r = await self._leader_query(MsgType.GET_FILE_NAMES_REQUEST, {"filepattern": pattern})
        return [] if r is None else r.payload.get("files", [])

    async def get_versions(self, name: str, n: int) -> List[Tuple[int, bytes]]:
        holders = await self.locate(name)
        vers = sorted({v for vs in holders.values() for v in vs})[-n:]
        out = []
        for v in reversed(vers):
            got = await self.fetch_from(holders, name, v)
            if got:
                out.append(got)
        return out

    async def announce_files(self) -> None:
        """Tell the (new) leader what this node holds (reference ALL_LOCAL_FILES, worker.py:593)."""
        leader = self.leader_fn()
        if leader and leader != self.me:
            await self.ep.send(leader, MsgType.ALL_LOCAL_FILES, {"all_files": self.local.all_files()})
        elif leader == self.me:
            self.meta.set_node_files(self.me, self.local.all_files())

    # ======================================================= leader handlers ==
    async def _l_put(self, fr: Frame) -> None:
        name = fr.payload["filename"]
        if self.meta.in_progress(name):
            await self.ep.reply(fr, MsgType.PUT_REQUEST_FAIL, {"filename": name, "error": "upload in progress"})
            return
        targets = self.meta.targets_for_put(name, self.storage_nodes())
        if not targets:
            await self.ep.reply(fr, MsgType.PUT_REQUEST_FAIL, {"filename": name, "error": "no storage nodes"})
            return
        version = self.meta.latest_version(name) + 1
        self.meta.begin(name, targets)
        req = {"filename": name, "version": version, "source": fr.sender, "token": fr.payload.get("token"),
               "source_blob": fr.payload.get("blob")}
        outcome = await self._fan_out(name, targets, req)
        self.meta.finish(name)
        if outcome == SUCCESS:
            await self.ep.reply(fr, MsgType.PUT_REQUEST_SUCCESS, {"filename": name, "version": version,
                                                                  "replicas": targets})
        else:
            await self.ep.reply(fr, MsgType.PUT_REQUEST_FAIL, {"filename": name, "error": "replica failed"})

    async def _fan_out(self, name: str, targets: List[str], req: dict) -> str:
        pending = list(targets)
        tried = set(targets)
        outcome = None
        while pending:
            rs = await asyncio.gather(*(self.ep.request(t, MsgType.DOWNLOAD_FILE, req, timeout=self.timeout)
                                        for t in pending))
            retry = []
            for t, r in zip(pending, rs):
                ok = r is not None and r.type == MsgType.DOWNLOAD_FILE_SUCCESS
                if r is not None:
                    self._learn_delta(t, r.payload)
                if not ok and not self.ml.is_alive(t):
                    # replica died mid-PUT: substitute another node
                    self.meta.requests.get(name, {}).pop(t, None)
                    subs = [n for n in self.meta.place(name, self.storage_nodes(), 64) if n not in tried]
                    if subs:
                        tried.add(subs[0])
                        self.meta.requests.setdefault(name, {})[subs[0]] = "Waiting"
                        retry.append(subs[0])
                    continue
                outcome = self.meta.update(name, t, ok) or outcome
            pending = retry
        st = self.meta.requests.get(name, {})
        if st and all(v == SUCCESS for v in st.values()):
            return SUCCESS
        return FAILED

    async def _request_unless_dead(self, t: str, mtype, payload: dict, poll_s: float = 0.05):
        """A request to replica ``t`` that gives up as soon as the membership confirms ``t``
        dead (None, as on a timeout) instead of waiting out the request timeout: a bundle
        PUT in flight when a rank dies is re-placed right after the failure detector's
        verdict, not ``timeout`` seconds later (measured: a 2-kill config-5 pass spent ~10 s
        of its 12 with batches waiting for PUTs to dead replicas)."""
        req = asyncio.ensure_future(self.ep.request(t, mtype, payload, timeout=self.timeout))
        while not req.done():
            if not self.ml.is_alive(t):
                req.cancel()
                return None
            await asyncio.wait({req}, timeout=poll_s)
        return req.result()

    async def _l_put_many(self, fr: Frame) -> None:
        """Leader side of put_many: per-file placement and versions as a single PUT,
        but one DOWNLOAD_MANY per replica node for all of its files; a replica that
        dies mid-PUT is replaced per file (as _fan_out)."""
        names = list(dict.fromkeys(fr.payload.get("files", [])))
        alive = self.storage_nodes()
        failed = [n for n in names if self.meta.in_progress(n)]
        todo: Dict[str, List[str]] = {}
        for n in names:
            if n in failed:
                continue
            t = self.meta.targets_for_put(n, alive)
            if not t:
                failed.append(n)
                continue
            todo[n] = t
        versions = {n: self.meta.latest_version(n) + 1 for n in todo}
        for n, t in todo.items():
            self.meta.begin(n, t)
        src = {"source": fr.sender, "token": fr.payload.get("token"), "source_blob": fr.payload.get("blob")}
        if fr.payload.get("spool"):
            src.update(spool=fr.payload["spool"], host=fr.payload.get("host"))
        tried = {n: set(t) for n, t in todo.items()}
        pending = {n: list(t) for n, t in todo.items()}
        while pending:
            per_node: Dict[str, List[str]] = {}
            for n, ts in pending.items():
                for t in ts:
                    per_node.setdefault(t, []).append(n)
            nodes = sorted(per_node)
            rs = await asyncio.gather(*(self._request_unless_dead(
                t, MsgType.DOWNLOAD_MANY, {"files": [[n, versions[n]] for n in per_node[t]], **src}) for t in nodes))
            pending = {}
            for t, r in zip(nodes, rs):
                got = r.payload.get("ok", {}) if r is not None else {}
                if r is not None:
                    self._learn_delta(t, {"files": got})
                dead = r is None and not self.ml.is_alive(t)
                for n in per_node[t]:
                    if n in got:
                        self.meta.update(n, t, True)
                        continue
                    if dead:  # replica died mid-PUT: substitute another node for this file
                        self.meta.requests.get(n, {}).pop(t, None)
                        subs = [x for x in self.meta.place(n, self.storage_nodes(), 64) if x not in tried[n]]
                        if subs:
                            tried[n].add(subs[0])
                            self.meta.requests.setdefault(n, {})[subs[0]] = "Waiting"
                            pending.setdefault(n, []).append(subs[0])
                            continue
                    self.meta.update(n, t, False)
        ok = []
        for n in todo:
            st = self.meta.requests.get(n, {})
            (ok if st and all(v == SUCCESS for v in st.values()) else failed).append(n)
            self.meta.finish(n)
        await self.ep.reply(fr, MsgType.PUT_MANY_REPLY, {"ok": ok, "failed": failed})

    async def _l_delete(self, fr: Frame) -> None:
        name = fr.payload["filename"]
        holders = list(self.meta.holders(name))
        if not holders:
            await self.ep.reply(fr, MsgType.DELETE_FILE_REQUEST_FAIL, {"filename": name, "error": "no such file"})
            return
        rs = await asyncio.gather(*(self.ep.request(h, MsgType.DELETE_FILE, {"filename": name}, timeout=self.timeout)
                                    for h in holders))
        ok = True
        for h, r in zip(holders, rs):
            if r is None:
                ok = ok and not self.ml.is_alive(h)
                continue
            self._learn_delta(h, r.payload)
            ok = ok and r.type == MsgType.DELETE_FILE_ACK
        await self.ep.reply(fr, MsgType.DELETE_FILE_REQUEST_SUCCESS if ok else MsgType.DELETE_FILE_REQUEST_FAIL,
                            {"filename": name})

    async def _wait_settled(self) -> None:
        """A listing arriving while this new leader still collects COORDINATE_ACKs waits for
        adopt() (bounded: a round whose acks never come answers from what it has)."""
        if not self._settled.is_set():
            try:
                await asyncio.wait_for(self._settled.wait(), min(self.timeout, 5.0))
            except asyncio.TimeoutError:
                pass

    async def _l_ls(self, fr: Frame) -> None:
        await self._wait_settled()
        name = fr.payload["filename"]
        await self.ep.reply(fr, MsgType.LIST_FILE_REQUEST_ACK, {"filename": name,
                                                                "machines": sorted(self.meta.holders(name))})

    async def _l_get(self, fr: Frame) -> None:
        name = fr.payload["filename"]
        await self.ep.reply(fr, MsgType.GET_FILE_REQUEST_ACK, {"filename": name,
                                                               "machineids_with_file_versions": self.meta.holders(name)})

    async def _l_ls_all(self, fr: Frame) -> None:
        await self._wait_settled()
        pat = fr.payload.get("filepattern", "*")
        await self.ep.reply(fr, MsgType.GET_FILE_NAMES_REQUEST_ACK, {"filepattern": pat,
                                                                     "files": self.meta.matching(pat)})

    async def _l_all_local_files(self, fr: Frame) -> None:
        self._learn(fr.sender, fr.payload.get("all_files", {}))

    async def _l_files_stored(self, fr: Frame) -> None:
        """A writer stored files on their replicas itself (put_many_direct): record them."""
        for node, files in fr.payload.get("files", {}).items():
            self._learn_delta(node, {"files": files})
        await self.ep.reply(fr, MsgType.FILES_STORED_ACK, {})

    def _learn_delta(self, node: str, payload: dict) -> None:
        """A replica's reply names only the files it just touched ("files": name ->
        its versions there now; the reference sent its whole listing with every
        reply, worker.py:143, which grows with every output file the service PUTs)."""
        files = payload.get("files")
        if files is None:  # a peer that still sends its full listing
            if "all_files" in payload:
                self._learn(node, payload["all_files"])
            return
        self.meta.update_node_files(node, files)
        if self._round is not None:
            rd = self._round.setdefault(node, {})
            for k, v in files.items():
                rd[k] = sorted(set(rd.get(k, [])) | {int(x) for x in v})

    def _learn(self, node: str, files: Dict[str, list]) -> None:
        """A node's current file list (announce / replica reply); while a
        COORDINATE round is open it is also kept aside for adopt()."""
        self.meta.set_node_files(node, files)
        if self._round is not None:
            self._round[node] = {k: list(v) for k, v in files.items()}

    def begin_round(self) -> None:
        """Election: this node starts a COORDINATE round (before sending it)."""
        self._round = {}
        self._settled.clear()

    def adopt(self, acks: Dict[str, dict]) -> None:
        """New leader: rebuild the file map from COORDINATE_ACK payloads.

        A node's ACK is its authoritative current list (files it deleted or
        evicted since are gone); only what that node reported AFTER the round
        started - an ALL_LOCAL_FILES announce or a PUT replica reply racing the
        ACKs - is unioned in. Nodes that did not ack keep the leader's earlier
        view; entries of nodes that are not alive are dropped."""
        fm = self.meta.file_map
        late = self._round or {}
        self._round = None
        for node in [n for n in fm if n != self.me and not self.ml.is_alive(n)]:
            fm.pop(node, None)
        self.meta.set_node_files(self.me, self.local.all_files())
        for node, p in acks.items():
            files = {k: set(int(x) for x in v) for k, v in p.get("all_files", {}).items()}
            for k, v in late.get(node, {}).items():
                files.setdefault(k, set()).update(int(x) for x in v)
            self.meta.set_node_files(node, {k: sorted(v) for k, v in files.items()})
        self._settled.set()

    async def node_failed(self, node: str) -> int:
        """Leader: drop the node's files and restore the replication factor."""
        if not self.is_leader():
            return 0
        self.meta.remove_node(node)
        plan = self.meta.under_replicated(self.storage_nodes())
        n = 0
        for name, src, new_nodes in plan:
            for t in new_nodes:
                r = await self.ep.request(t, MsgType.REPLICATE_FILE, {"filename": name, "source": src},
                                          timeout=self.timeout)
                if r is not None and r.type == MsgType.REPLICATE_FILE_SUCCESS:
                    self._learn_delta(t, r.payload)
                    n += 1
        return n

    # ====================================================== replica handlers ==
    async def _r_download(self, fr: Frame) -> None:
        p = fr.payload
        try:
            items = await self.blobs.fetch(p["source"], {"op": "outbox", "token": p.get("token")},
                                           addr=p.get("source_blob"))
            if not items:
                raise FileNotFoundError("outbox empty")
            self.local.put_bytes(p["filename"], items[0][1], version=p.get("version"))
            mt = MsgType.DOWNLOAD_FILE_SUCCESS
        except (ConnectionError, OSError, asyncio.TimeoutError) as e:
            log.warning("%s: download %s failed: %s", self.me, p["filename"], e)
            mt = MsgType.DOWNLOAD_FILE_FAIL
        await self.ep.reply(fr, mt, {"filename": p["filename"], "files": self._delta(p["filename"])})

    def _delta(self, name: str) -> Dict[str, List[int]]:
        return {name: self.local.versions(name)}

    def _link_from_spool(self, spool: str, files: List[Tuple[str, int]]) -> Dict[str, List[int]]:
        done = self.local.put_links([(n, os.path.join(spool, n), v) for n, v in files])
        return {n: self.local.versions(n) for n in done}

    async def _r_download_many(self, fr: Frame) -> None:
        p = fr.payload
        # version 0 (put_many_direct): this replica assigns the next version of the name
        files = [(n, int(v) if int(v) > 0 else None) for n, v in p.get("files", [])]
        ok: Dict[str, List[int]] = {}
        loop = asyncio.get_running_loop()
        spool = p.get("spool")
        if spool and p.get("host") == HOST_ID:
            try:  # same machine: one hard link per file, no bytes moved (a few us each: inline,
                # an executor hand-off would cost more GIL round trips than the syscalls)
                ok = self._link_from_spool(spool, files)
                self.linked += len(ok)
            except OSError as e:  # another filesystem / spool gone: pull the bytes instead
                log.info("%s: spool link failed (%s); pulling over the blob plane", self.me, e)
                ok = {}
        if len(ok) < len(files):
            # only the files no link stored: a linked file pulled again would be stored twice
            # (twice the version count on the leaderless path, where this replica numbers them)
            missing = [(n, v) for n, v in files if n not in ok]
            req = {"op": "outbox_many", "token": p.get("token"), "names": [n for n, _ in missing]}
            try:
                if p["source"] == self.me:  # this node PUT the bundle: take it from its own outbox
                    items = self.source.read(req)
                else:
                    items = await self.blobs.fetch(p["source"], req, addr=p.get("source_blob"))
                if len(items) == len(missing):
                    def write():
                        for (n, v), (_, data) in zip(missing, items):
                            self.local.put_bytes(n, data, version=v)
                            ok[n] = self.local.versions(n)
                    await loop.run_in_executor(None, write)  # file writes never block the SWIM loop
                    self.pulled += len(missing)
            except (ConnectionError, OSError, asyncio.TimeoutError) as e:
                log.warning("%s: download of %d files failed: %s", self.me, len(files), e)
        await self.ep.reply(fr, MsgType.DOWNLOAD_MANY_REPLY,
                            {"ok": ok, "failed": [n for n, _ in files if n not in ok]})

    async def _r_delete(self, fr: Frame) -> None:
        ok = self.local.delete(fr.payload["filename"])
        await self.ep.reply(fr, MsgType.DELETE_FILE_ACK if ok else MsgType.DELETE_FILE_NAK,
                            {"filename": fr.payload["filename"], "files": self._delta(fr.payload["filename"])})

    async def _r_replicate(self, fr: Frame) -> None:
        p = fr.payload
        try:
            items = await self.blobs.fetch(p["source"], {"op": "get_all", "name": p["filename"]})
            for v, data in items:
                self.local.put_bytes(p["filename"], data, version=v)
            mt = MsgType.REPLICATE_FILE_SUCCESS if items else MsgType.REPLICATE_FILE_FAIL
        except (ConnectionError, OSError, asyncio.TimeoutError):
            mt = MsgType.REPLICATE_FILE_FAIL
        await self.ep.reply(fr, mt, {"filename": p["filename"], "files": self._delta(p["filename"])})
