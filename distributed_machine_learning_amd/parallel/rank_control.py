"""This rank's host control plane (UDP, never RCCL) for the collective service.

Reference: every VM ran the failure detector, the SDFS replica, the leader's
handlers and the CLI in one asyncio process (worker.py:2036-2044, 887-1059).
Here each GPU rank runs a cluster Node with role "rank" in a daemon thread with
its own event loop; the serve loop (parallel/service.py) talks to it through
thread-safe hooks.
"""
from __future__ import annotations

import asyncio
import logging
import threading
import time
from typing import Callable, Dict, List, Optional

from ..serving.jobs import Batch
from .rank_backend import split_version, synthetic_names
from ..cluster.tasks import spawn

log = logging.getLogger(__name__)


class RankControl:
    """This rank's host control plane, in a daemon thread with its own asyncio
    loop: a cluster Node with role "rank" (SWIM membership -> dead ranks for the
    elastic group, bully election -> store leader = coordinator, the replicated
    store with its TCP blob plane) plus the job-service request handlers the
    reference leader served (SUBMIT_JOB_REQUEST, C1, C2, C3 = SET_BATCH_SIZE,
    C5 = GET_ASSIGNMENTS, JOB_STATUS; worker.py:887-1059). Requests reach the
    serve loop through its inbox; replies go out once the request's log record
    has been broadcast (committed on every rank)."""

    def __init__(self, grank: int, world: int, base_port: int, store_dir: str, host: str = "127.0.0.1",
                 period: float = 0.1, ping_timeout: float = 0.1, suspect_timeout: float = 1.5,
                 replication: int = 4, on_dead: Optional[Callable[[int], None]] = None,
                 on_alive: Optional[Callable[[int], None]] = None, rejoin: bool = False):
        self.grank, self.world, self.base, self.host = grank, world, base_port, host
        self.store_dir, self.replication = store_dir, replication
        self.period, self.ping_timeout, self.suspect_timeout = period, ping_timeout, suspect_timeout
        self.on_dead, self.on_alive, self.rejoin = on_dead, on_alive, rejoin
        self.svc = None  # the CollectiveService it serves
        self.loop_lag_max = 0.0  # the longest this thread's event loop was late for a 20 ms timer, s
        self.put_lat: List[float] = []  # output bundle PUT latencies (call -> every replica stored), s
        # output bundles spooled once for same-machine replicas (hard links, store/service.py);
        # DML_SPOOL_OUTPUTS=0: every replica pulls over the blob plane (A/B)
        import os

        self.spool_outputs = os.environ.get("DML_SPOOL_OUTPUTS", "1") != "0"
        # outputs are PUT leaderless (store.service.put_many_direct: the writer fans out to the
        # replicas, one FILES_STORED message to the leader); DML_DIRECT_PUTS=0: through the leader
        self.direct_puts = os.environ.get("DML_DIRECT_PUTS", "1") != "0"
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.node = None
        self.ready = threading.Event()
        self.dead: set = set()
        self.thread = threading.Thread(target=self._main, daemon=True, name=f"rank-control-{grank}")

    def addr(self, g: int) -> str:
        return f"{self.host}:{self.base + g}"

    def rank_of(self, name: str) -> Optional[int]:
        try:
            return int(name.rsplit(":", 1)[1]) - self.base
        except (ValueError, IndexError):
            return None

    async def _lag_monitor(self, tick: float = 0.02) -> None:
        """How late the loop runs a timer: SWIM acks share this loop with the store's request
        handlers, so a handler that holds it past the suspicion timeout gets this rank declared
        dead while it is alive."""
        while True:
            t = time.perf_counter()
            await asyncio.sleep(tick)
            self.loop_lag_max = max(self.loop_lag_max, time.perf_counter() - t - tick)

    # ------------------------------------------------------------ thread --
    def start(self, timeout: float = 30.0) -> "RankControl":
        import atexit

        atexit.register(self.stop)  # never tear the loop down with its tasks pending (see fd_thread)
        self.thread.start()
        if not self.ready.wait(timeout):
            raise RuntimeError("rank control plane did not start")
        return self

    def _main(self) -> None:
        self.loop = asyncio.new_event_loop()
        asyncio.set_event_loop(self.loop)
        self._task = spawn(self._run(), self.loop)
        self.loop.run_forever()
        pending = [t for t in asyncio.all_tasks(self.loop) if not t.done()]
        for t in pending:
            t.cancel()
        if pending:
            self.loop.run_until_complete(asyncio.gather(*pending, return_exceptions=True))
        self.loop.close()

    async def _run(self) -> None:
        from ..cluster.frames import MsgType
        from ..serving.node import Node, NodeConfig

        cfg = NodeConfig(host=self.host, port=self.base + self.grank, role="rank", seeds=[self.addr(0)],
                         store_dir=self.store_dir, period=self.period, ping_timeout=self.ping_timeout,
                         suspect_timeout=self.suspect_timeout, cleanup_time=30.0, replication=self.replication,
                         meta={"prio": self.grank, "rank": self.grank})
        self.node = n = await Node(cfg).start()
        spawn(self._lag_monitor(), self.loop)
        on = n.ep.on
        on(MsgType.SUBMIT_JOB_REQUEST, self._on_submit)
        on(MsgType.SET_BATCH_SIZE, self._on_batch_size)
        on(MsgType.GET_C1_COMMAND, self._on_c1)
        on(MsgType.GET_C2_COMMAND, self._on_c2)
        on(MsgType.GET_ASSIGNMENTS, self._on_c5)
        on(MsgType.JOB_STATUS, self._on_status)
        on(MsgType.GET_OUTPUT, self._on_get_output)
        on(MsgType.FETCH_INTRODUCER, self._on_fetch_leader)   # every rank is an introducer for clients
        n.ml.on_fail.append(self._member_failed)
        n.ml.on_join.append(self._member_joined)
        await n.join()
        # every rank knows the static job membership: once all have joined, the
        # bully election settles on the highest rank (= the collective
        # coordinator); serving starts only then, so store requests of the first
        # steps already reach the right leader
        want = self.addr(self.world - 1)
        if self.rejoin:  # a restarted rank: the running job's leader stays; learn it by joining
            for _ in range(200):
                if n.leader() is not None:
                    break
                await asyncio.sleep(0.05)
            self.ready.set()
            return
        for _ in range(400):
            if len([m for m in n.ml.alive() if (n.ml.get(m).meta or {}).get("role") == "rank"]) >= self.world:
                break
            await asyncio.sleep(0.05)
        for _ in range(400):
            if n.leader() == want:
                break
            if not n.election.in_election:
                n.election.trigger()
            await asyncio.sleep(0.05)
        self.ready.set()

    def _member_failed(self, name: str) -> None:
        g = self.rank_of(name)
        if g is not None and 0 <= g < self.world and g not in self.dead:
            self.dead.add(g)
            log.warning("rank %d: SWIM confirmed rank %d dead", self.grank, g)
            if self.on_dead is not None:
                self.on_dead(g)

    def _member_joined(self, name: str) -> None:
        """SWIM: a rank that had died is alive again (a restarted process)."""
        g = self.rank_of(name)
        if g is not None and 0 <= g < self.world and g in self.dead:
            self.dead.discard(g)
            log.warning("rank %d: SWIM saw rank %d rejoin", self.grank, g)
            if self.on_alive is not None:
                self.on_alive(g)

    def stop(self) -> None:
        if self.loop is None or not self.thread.is_alive():
            return

        async def _shutdown():
            try:
                await self.node.stop()
            except Exception:
                pass
            tasks = [t for t in asyncio.all_tasks() if t is not asyncio.current_task()]
            for t in tasks:
                t.cancel()
            await asyncio.gather(*tasks, return_exceptions=True)
        try:
            asyncio.run_coroutine_threadsafe(_shutdown(), self.loop).result(timeout=5)
        except Exception:
            pass
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.thread.join(timeout=5)

    # ------------------------------------------------------- serve hooks --
    def attach(self, svc) -> None:
        self.svc = svc

    def call(self, coro, timeout: float = 30.0):
        """Run a coroutine on the control loop from the serve thread."""
        return asyncio.run_coroutine_threadsafe(coro, self.loop).result(timeout)

    def committed(self, replies: List[Optional[Callable]], results: List[dict]) -> None:
        for cb, r in zip(replies, results):
            if cb is not None:
                self.loop.call_soon_threadsafe(cb, r)

    def jobs_progress(self, batches: List[Batch]) -> None:
        """Tell requesters whose job just finished (SUBMIT_JOB_REQUEST_SUCCESS)."""
        from ..cluster.frames import MsgType

        seen = set()
        for b in batches:
            j = self.svc.coord.jobs.jobs.get(b.job_id)
            if j is not None and j.done and j.job_id not in seen and ":" in j.requester:  # a node, not "local"
                seen.add(j.job_id)
                self.loop.call_soon_threadsafe(
                    lambda jj=j: spawn(
                        self.node.ep.send(jj.requester, MsgType.SUBMIT_JOB_REQUEST_SUCCESS, {"jobid": jj.job_id}),
                        self.loop))

    def became_coordinator(self, previous: int) -> None:
        log.warning("rank %d: now the coordinator (was rank %d)", self.grank, previous)
        # requesters of jobs that finished while the old coordinator was dying are told again
        done = [j for j in self.svc.coord.jobs.jobs.values() if j.done]
        self.jobs_progress([Batch(j.job_id, 0, j.model, []) for j in done])

    def store_put(self, name: str, data: bytes, deadline_s: float = 60.0) -> None:
        """PUT into the store, retried across a store-leader change (the leader
        is the coordinator rank, which is what fails over)."""
        t0, err = time.monotonic(), ""
        while time.monotonic() - t0 < deadline_s:
            try:
                ok, err = self.call(self.node.store.put(data, name), timeout=30)
            except Exception as e:  # leader unreachable mid-failover
                ok, err = False, str(e)
            if ok:
                return
            time.sleep(0.1)
        raise RuntimeError(f"store put {name}: {err}")

    def store_put_many_async(self, items, done: Callable[[List[str], List[str]], None],
                             deadline_s: float = 60.0, attempt_s: float = 8.0) -> None:
        """PUT a bundle of files (store.service.put_many: one leader round trip) without
        blocking the caller; files the store refused are retried (a store-leader change
        mid-PUT; each attempt bounded by ``attempt_s``) until ``deadline_s``.
        ``done(stored, failed)`` runs on the control loop. The bundle is first written
        once into a spool directory by the CALLING thread (the output writer), so the
        replicas on this machine hard-link it (store/service.py) and no byte of it crosses
        the control loop; a spool failure falls back to the blob plane."""
        import shutil

        spool = None
        if self.spool_outputs:
            try:
                spool = self.node.store.spool(items)
            except OSError as e:
                log.warning("rank %d: output spool failed (%s); replicas pull over the blob plane", self.grank, e)

        t_call = time.monotonic()

        async def go():
            remaining = dict(items)
            stored: List[str] = []
            t0, err = time.monotonic(), ""
            while remaining and time.monotonic() - t0 < deadline_s:
                try:  # one attempt is bounded: a leader that died mid-PUT must not eat the deadline
                    put = self.node.store.put_many_direct if self.direct_puts else self.node.store.put_many
                    ok, _, err = await asyncio.wait_for(put(list(remaining.items()), spool=spool), attempt_s)
                except Exception as e:  # leader unreachable mid-failover
                    ok, err = [], str(e)
                for n in ok:
                    if remaining.pop(n, None) is not None:
                        stored.append(n)
                if remaining:
                    await asyncio.sleep(0.1)
            if remaining:
                log.error("rank %d: store put of %d files failed: %s", self.grank, len(remaining), err)
            if spool is not None:  # every replica linked its copy (or pulled it): the spool entries go
                self.loop.run_in_executor(None, shutil.rmtree, spool, True)
            self.put_lat.append(time.monotonic() - t_call)
            try:
                done(stored, list(remaining))
            except Exception:
                log.exception("rank %d: bundle completion callback failed", self.grank)
        asyncio.run_coroutine_threadsafe(go(), self.loop)

    def store_loader(self, names: List[str]) -> Dict[str, Optional[bytes]]:
        """Fetch store images; ``name@v`` is that version exactly (pinned at submit). The
        versions this node holds are read in the calling thread by one native batch
        (store/fastio.read_many); only the rest go through the control loop."""
        from ..store import fastio

        local = self.node.local
        out: Dict[str, Optional[bytes]] = {}
        here, miss = [], []
        for nm in names:
            base, ver = split_version(nm)
            (here if local.has(base, ver) else miss).append((nm, base, ver))
        if here:
            try:
                blobs = fastio.read_many([local.path(b, v) for _, b, v in here])
                out.update((nm, blob) for (nm, _, _), blob in zip(here, blobs))
            except OSError:   # a version removed under us: the control loop sorts it out
                miss += here
        if not miss:
            return out
        names = [nm for nm, _, _ in miss]

        async def fetch_all():
            sem = asyncio.Semaphore(16)

            async def one(nm):
                base, ver = split_version(nm)
                async with sem:
                    if self.node.local.has(base, ver):
                        return nm, self.node.local.get_bytes(base, ver)
                    got = await self.node.store.get(base, ver)
                    return nm, None if got is None else got[1]
            return dict(await asyncio.gather(*(one(nm) for nm in names)))
        out.update(self.call(fetch_all(), timeout=120))
        return out

    def pin_versions(self, names: List[str]) -> List[str]:
        """(coordinator, control thread) name -> name@latest-version from the
        store metadata, so every rank reads the same bytes for the whole job
        (reference: the latest version at task time, worker.py:1323-1366)."""
        meta = self.node.store.meta
        out = []
        for nm in names:
            v = meta.latest_version(nm)
            out.append(f"{nm}@{v}" if v and v > 0 else nm)
        return out

    # ----------------------------------------------------------- handlers --
    async def _on_fetch_leader(self, fr) -> None:
        """Reference FETCH_INTRODUCER (introduce process/worker.py:55-58): any rank
        tells a client who leads, once the election has settled."""
        from ..cluster.frames import MsgType

        if self.ready.is_set() and self.node.leader() is not None:
            await self.node.ep.reply(fr, MsgType.FETCH_INTRODUCER_ACK, {"introducer": self.node.leader()})

    def _active(self) -> bool:
        return self.svc is not None and self.svc.is_coordinator()

    async def _on_submit(self, fr) -> None:
        from ..cluster.frames import MsgType

        if not self._active():
            return  # not the coordinator: the client retries at the elected leader
        p = fr.payload
        model = p["model"]
        n = int(p["images_count"])
        if p.get("synthetic"):
            names = synthetic_names(n)
        else:
            from ..serving.jobs import pick_images

            names = self.pin_versions(pick_images(sorted(self.node.store.meta.matching("*.jpeg")), n))

        def reply(res, fr=fr):
            spawn(self.node.ep.reply(fr, MsgType.SUBMIT_JOB_REQUEST_ACK, res), self.loop)
            if res.get("batches") == 0:
                spawn(self.node.ep.send(fr.sender, MsgType.SUBMIT_JOB_REQUEST_SUCCESS,
                                                        {"jobid": res["jobid"]}))
        self.svc.submit_local(model, images=names, requester=fr.sender, reply=reply)

    async def _on_batch_size(self, fr) -> None:
        from ..cluster.frames import MsgType

        if not self._active():
            return

        def reply(res, fr=fr):
            if fr.seq:
                spawn(self.node.ep.reply(fr, MsgType.SET_BATCH_SIZE_ACK, res), self.loop)
        self.svc.set_batch_size(fr.payload["model"], int(fr.payload["batch_size"]), reply=reply)

    async def _on_c1(self, fr) -> None:
        from ..cluster.frames import MsgType

        if self._active():
            with self.svc.coord.lock:
                c1 = self.svc.coord.metrics.c1()
            await self.node.ep.reply(fr, MsgType.GET_C1_COMMAND_ACK, {"c1": c1})

    async def _on_c2(self, fr) -> None:
        from ..cluster.frames import MsgType

        if self._active():
            with self.svc.coord.lock:
                p = self.svc.coord.metrics.c2_reference_payload()
                p["detail"] = self.svc.coord.metrics.c2()
            await self.node.ep.reply(fr, MsgType.GET_C2_COMMAND_ACK, p)

    async def _on_c5(self, fr) -> None:
        from ..cluster.frames import MsgType

        if self._active():
            p = fr.payload or {}
            with self.svc.coord.lock:
                a = self.svc.coord.assignments()
                h = self.svc.coord.recent(int(p.get("history", 16)), p.get("job_id"))
            await self.node.ep.reply(fr, MsgType.GET_ASSIGNMENTS_ACK, {"assignments": a, "history": h})

    async def _on_get_output(self, fr) -> None:
        """get-output at the coordinator: final_<job>.json rendered once from the top-5 rows the
        service gathered over the data group (CollectiveService.final_output), stored in the
        replicated store; the requester fetches it by name. {"name": None} (not the coordinator,
        or a batch of the job not gathered here, e.g. after a fail-over): the requester merges
        the output files instead (the reference's get-output, worker.py:1617-1627)."""
        from ..cluster.frames import MsgType

        if not self._active() or self.svc is None:
            await self.node.ep.reply(fr, MsgType.GET_OUTPUT_ACK, {"name": None})
            return
        jid = int(fr.payload["jobid"])
        tag = self.svc.writer.host_tag if getattr(self.svc, "writer", None) is not None else "node"
        loop = asyncio.get_running_loop()
        data = await loop.run_in_executor(None, self.svc.final_output, jid, tag, 5.0)   # native render, GIL released
        name = None
        if data is not None:
            name = f"final_{jid}.json"
            ok, _ = await self.node.store.put(data, name)
            name = name if ok else None
        await self.node.ep.reply(fr, MsgType.GET_OUTPUT_ACK, {"name": name})

    async def _on_status(self, fr) -> None:
        from ..cluster.frames import MsgType

        if not self._active():
            return
        with self.svc.coord.lock:
            j = self.svc.coord.jobs.jobs.get(int(fr.payload["jobid"]))
            st = {"jobid": fr.payload["jobid"], "known": j is not None, "done": bool(j and j.done),
                  "batches_done": j.batches_done if j else 0, "batches_total": j.batches_total if j else 0}
        await self.node.ep.reply(fr, MsgType.JOB_STATUS_ACK, st)
