"""A cluster node: composition of every control-plane role.

Reference: one ``Worker`` god object per VM (worker.py:29-2044) holding FD,
SDFS client/replica, leader duties, scheduler, inference worker, metrics and
CLI, glued by a ``Global`` service locator (globalClass.py). Roles were fixed
by hostname (H1 leader, H2 standby, H3..H10 workers; worker.py:52,
election.py:27).

Here the roles are explicit components wired by this class, and the role comes
from configuration (``coordinator`` / ``standby`` / ``worker`` / ``client``);
coordinator-eligible nodes each hold a Coordinator object that is active only
while that node is the elected leader.
"""
from __future__ import annotations

import asyncio
import logging
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..cluster.election import Election
from ..cluster.failure_detector import FailureDetector
from ..cluster.frames import Frame, MsgType
from ..cluster.introducer import fetch_leader, update_leader
from ..cluster.membership import MembershipList
from ..cluster.transport import Endpoint, LoopbackNetwork, UdpTransport
from ..store.blob import BlobServer, BlobSource, InProcBlobNetwork, TcpBlobClient
from ..store.local_store import LocalFileStore
from ..store.service import StoreService
from .coordinator import Coordinator
from .journal import open_journal
from .inference import Backend, make_backend
from .worker import WorkerRole
from ..cluster.tasks import spawn

log = logging.getLogger(__name__)


@dataclass
class NodeConfig:
    host: str = "127.0.0.1"
    port: int = 0
    role: str = "worker"                 # coordinator | standby | worker | client | rank
    # "rank": one GPU process of the RCCL collective service (parallel/service.py):
    # coordinator-eligible store node whose job service is the replicated
    # collective coordinator, so no host Coordinator / WorkerRole is created here
    introducer: Optional[str] = None     # DNS "host:port" (reference config.py:25-26)
    seeds: List[str] = field(default_factory=list)
    store_dir: str = "/tmp/dml_store"
    out_dir: Optional[str] = None
    backend: str = "cpu"                 # gpu | cpu | fake
    backend_kw: Dict = field(default_factory=dict)
    testing: bool = False                # reference -t: 3 % send drop + meters
    drop_rate: float = 0.03
    period: float = 0.5                  # FD period (reference 12 s / README 2.5 s)
    ping_timeout: float = 0.25           # (reference 10 s / 2 s)
    suspect_timeout: float = 2.0
    cleanup_time: float = 10.0           # (reference 30 s / 10 s)
    replication: int = 4
    batch_sizes: Dict[str, int] = field(default_factory=lambda: {"ResNet50": 10, "InceptionV3": 10})
    store_timeout: float = 10.0
    journal: Optional[str] = None        # coordinator job journal (restart recovery), serving/journal.py
    meta: Dict = field(default_factory=dict)  # extra membership metadata (e.g. the global rank)


class Node:
    def __init__(self, cfg: NodeConfig, net: Optional[LoopbackNetwork] = None,
                 blob_net: Optional[InProcBlobNetwork] = None, name: Optional[str] = None,
                 backend: Optional[Backend] = None):
        self.cfg = cfg
        self.net, self.blob_net = net, blob_net
        self._name = name
        self._backend = backend
        self.job_done: Dict[int, asyncio.Event] = {}
        self.last_output_fast = False    # the last get_output came from the coordinator's gathered results
        self.started_at = time.monotonic()

    # ---------------------------------------------------------------- start --
    async def start(self) -> "Node":
        cfg = self.cfg
        if self.net is not None:
            t = self.net.transport(self._name or f"{cfg.host}:{cfg.port}")
        else:
            t = await UdpTransport(cfg.host, cfg.port, drop_rate=cfg.drop_rate if cfg.testing else 0.0).start()
        self.transport = t
        self.name = t.name
        self.ep = Endpoint(t)
        self.local = LocalFileStore(os.path.join(cfg.store_dir, self.name.replace(":", "_")))
        self.source = BlobSource(self.local)
        meta = {"role": cfg.role, "eligible": cfg.role in ("coordinator", "standby", "rank")}
        meta.update(cfg.meta)
        if self.blob_net is not None:
            self.blob_net.register(self.name, self.source)
            self.blobs = self.blob_net
            self.blob_server = None
        else:
            self.blob_server = await BlobServer(self.source, cfg.host).start()
            meta["blob"] = self.blob_server.addr
            self.blobs = TcpBlobClient(lambda n: (self.ml.get(n).meta.get("blob") if self.ml.get(n) else None))
        self.ml = MembershipList(self.name, suspect_timeout=cfg.suspect_timeout, cleanup_time=cfg.cleanup_time,
                                 meta=meta)
        self.fd = FailureDetector(self.ep, self.ml, period=cfg.period, ping_timeout=cfg.ping_timeout)
        self.election = Election(self.ep, self.ml, timeout=max(0.2, cfg.ping_timeout * 2),
                                 ack_payload=lambda: {"all_files": self.local.all_files()},
                                 on_elected=self._on_elected, on_new_leader=self._on_new_leader)
        storage = lambda n: (self.ml.get(n) is not None and self.ml.get(n).meta.get("role") != "client")
        self.store = StoreService(self.ep, self.ml, self.local, self.source, self.blobs, self.leader,
                                  replication=cfg.replication, timeout=cfg.store_timeout, storage_role=storage)
        self.election.on_round_start = self.store.begin_round
        self.coordinator: Optional[Coordinator] = None
        if meta["eligible"] and cfg.role != "rank":
            self.coordinator = Coordinator(self.ep, self.ml, list_images=self.store.meta.matching,
                                           locate=self.store.meta.holders, batch_sizes=dict(cfg.batch_sizes),
                                           is_active=lambda: self.is_leader(), journal=open_journal(cfg.journal))
        self.worker: Optional[WorkerRole] = None
        if cfg.role == "worker":
            be = self._backend or make_backend(cfg.backend, **cfg.backend_kw)
            self.worker = WorkerRole(self.ep, self.store, be, self.leader, self.name.replace(":", "_"),
                                     out_dir=cfg.out_dir)
        self.ep.on(MsgType.SUBMIT_JOB_REQUEST_SUCCESS, self._on_job_success)
        # a rank-service RankControl replaces this with its gathered-results fast path
        self.ep.on(MsgType.GET_OUTPUT, self._on_get_output)
        self.ml.on_fail.append(self._on_member_failed)
        self.ml.on_join.append(self._on_member_joined)
        self.ep.start()
        return self

    async def join(self) -> None:
        """Reference join flow (worker.py:572-596, 1137-1148): ask the introducer
        DNS who leads; become leader if nobody / me, else INTRODUCE to the leader."""
        leader = None
        if self.cfg.introducer:
            leader = await fetch_leader(self.ep, self.cfg.introducer)
        if leader is None and self.cfg.seeds:
            leader = next((sd for sd in self.cfg.seeds if sd != self.name), None)
        if leader is None or leader == self.name:
            if self.coordinator is not None:
                self.election.set_leader(self.name)
                self.store.meta.set_node_files(self.name, self.local.all_files())
        else:
            ok = await self.fd.join(leader)
            if not ok:
                log.warning("%s: join via %s failed", self.name, leader)
            self.election.set_leader(leader)
            await self.store.announce_files()
        self.fd.start()

    async def stop(self) -> None:
        self.fd.stop()
        self.ep.stop()
        if self.blob_server:
            self.blob_server.close()

    # ------------------------------------------------------------- queries --
    def leader(self) -> Optional[str]:
        return self.election.leader

    def is_leader(self) -> bool:
        return self.election.leader == self.name

    # ----------------------------------------------------------- callbacks --
    def _on_member_failed(self, name: str) -> None:
        self.election.leader_failed(name)
        if self.is_leader():
            if self.coordinator is not None:
                self.coordinator.worker_failed(name)
            spawn(self.store.node_failed(name))

    def _on_member_joined(self, name: str) -> None:
        if self.is_leader() and self.coordinator is not None:
            spawn(self.coordinator.schedule())

    def _on_elected(self, acks: Dict[str, dict]) -> None:
        self.store.adopt(acks)
        if self.coordinator is not None:
            self.coordinator.take_over()

    def _on_new_leader(self, leader: str) -> None:
        loop = asyncio.get_running_loop()
        if leader == self.name:
            if self.cfg.introducer:
                spawn(update_leader(self.ep, self.cfg.introducer, self.name), loop)
            if self.coordinator is not None:
                spawn(self.coordinator.schedule(), loop)
        else:
            spawn(self.store.announce_files(), loop)

    async def _on_job_success(self, fr: Frame) -> None:
        jid = int(fr.payload["jobid"])
        self.job_done.setdefault(jid, asyncio.Event()).set()

    async def _on_get_output(self, fr: Frame) -> None:
        await self.ep.reply(fr, MsgType.GET_OUTPUT_ACK, {"name": None})

    # ------------------------------------------------------------- client --
    async def submit_job(self, model: str, n_images: int, timeout: float = 5.0) -> Optional[int]:
        leader = self.leader()
        if leader is None:
            return None
        r = await self.ep.request(leader, MsgType.SUBMIT_JOB_REQUEST, {"model": model, "images_count": n_images},
                                  timeout=timeout, retries=1)
        if r is None:
            return None
        jid = int(r.payload["jobid"])
        self.job_done.setdefault(jid, asyncio.Event())
        return jid

    async def wait_job(self, jid: int, timeout: float = 60.0) -> bool:
        ev = self.job_done.setdefault(jid, asyncio.Event())
        try:
            await asyncio.wait_for(ev.wait(), timeout)
            return True
        except asyncio.TimeoutError:
            return False

    async def leader_request(self, mtype: MsgType, payload: Optional[dict] = None, timeout: float = 3.0):
        leader = self.leader()
        if leader is None:
            return None
        return await self.ep.request(leader, mtype, payload or {}, timeout=timeout, retries=1)

    async def get_output(self, jid: int, dest_dir: str) -> Optional[str]:
        """Reference get-output (worker.py:1617-1627): ls-all output_<job>_*.json,
        fetch all, merge into final_<job>.json. Under the rank service the coordinator
        already holds every batch's top-5 (gathered over the data group) and returns the
        store name of final_<job>.json rendered from them; the merge here is the fallback."""
        os.makedirs(dest_dir, exist_ok=True)
        path = os.path.join(dest_dir, f"final_{jid}.json")
        # the rank service's coordinator renders final_<job>.json once from the results it
        # gathered (RankControl GET_OUTPUT); anything else answers None: merge the files here
        leader = self.leader()
        if leader is not None:
            r = await self.ep.request(leader, MsgType.GET_OUTPUT, {"jobid": jid}, timeout=self.store.timeout)
            name = r.payload.get("name") if r is not None else None
            if name:
                got = await self.store.get(name)
                if got:
                    with open(path, "wb") as f:
                        f.write(got[1])
                    self.last_output_fast = True
                    return path
        self.last_output_fast = False
        return await self.merge_output_files(jid, path)

    async def merge_output_files(self, jid: int, path: str) -> Optional[str]:
        import json

        from .output import merge_outputs

        names = await self.store.ls_all(f"output_{jid}_*.json")
        docs = []
        for n in names:
            got = await self.store.get(n)
            if got:
                docs.append(json.loads(got[1]))
        if not docs:
            return None
        with open(path, "w") as f:
            json.dump(merge_outputs(docs), f, indent=4)
        return path
