"""Replicated versioned store (SDFS equivalent): local versions, placement,
PUT/GET/DELETE/LS/LS-ALL/GET-VERSIONS, failure re-replication, TCP blobs."""
import asyncio

import pytest

from distributed_machine_learning_amd.cluster.membership import MembershipList
from distributed_machine_learning_amd.cluster.transport import Endpoint, LoopbackNetwork
from distributed_machine_learning_amd.store.blob import BlobServer, BlobSource, InProcBlobNetwork, TcpBlobClient
from distributed_machine_learning_amd.store.local_store import LocalFileStore
from distributed_machine_learning_amd.store.metadata import FAILED, SUCCESS, StoreMetadata
from distributed_machine_learning_amd.store.service import StoreService


def test_local_versions_capped_and_reloaded(tmp_path):
    s = LocalFileStore(str(tmp_path))
    for i in range(7):
        assert s.put_bytes("a.jpeg", bytes([i])) == i + 1
    assert s.versions("a.jpeg") == [3, 4, 5, 6, 7]
    assert s.get_bytes("a.jpeg") == bytes([6]) and s.get_bytes("a.jpeg", 3) == bytes([2])
    s2 = LocalFileStore(str(tmp_path))  # index rebuilt from disk (file_service.py:16-33)
    assert s2.versions("a.jpeg") == [3, 4, 5, 6, 7]
    assert s2.delete("a.jpeg") and not s2.has("a.jpeg")


def test_placement_bounded_and_deterministic():
    m = StoreMetadata(4)
    nodes = [f"n{i}" for i in range(8)]
    p = m.place("x.jpeg", nodes)
    assert len(set(p)) == 4 and p == m.place("x.jpeg", list(reversed(nodes)))
    assert len(m.place("x.jpeg", nodes[:2])) == 2  # reference looped forever here (leader.py:60)
    m.begin("x.jpeg", p)
    assert m.update("x.jpeg", p[0], True) is None
    assert m.update("x.jpeg", p[1], False) == FAILED  # failures are reported (leader.py:132 typo)


def _mk(net, blobs, tmp_path, names, leader="n0"):
    nodes = {}
    for n in names:
        ep = Endpoint(net.transport(n))
        ml = MembershipList(n, incarnation=1)
        ml.merge({o: [1, 1, {}] for o in names})
        local = LocalFileStore(str(tmp_path / n))
        src = BlobSource(local)
        blobs.register(n, src)
        svc = StoreService(ep, ml, local, src, blobs, lambda: leader, timeout=1.0)
        ep.start()
        nodes[n] = svc
    return nodes


def test_put_get_delete_ls(tmp_path):
    async def main():
        net, blobs = LoopbackNetwork(), InProcBlobNetwork()
        names = [f"n{i}" for i in range(6)]
        nodes = _mk(net, blobs, tmp_path, names)
        c = nodes["n5"]
        ok, err = await c.put(b"hello", "1.jpeg")
        assert ok, err
        holders = await c.ls("1.jpeg")
        assert len(holders) == 4
        ok, _ = await c.put(b"hello2", "1.jpeg")
        assert ok
        got = await nodes["n3"].get("1.jpeg")
        assert got == (2, b"hello2")
        vers = await c.get_versions("1.jpeg", 2)
        assert [v for v, _ in vers] == [2, 1] and vers[1][1] == b"hello"
        await c.put(b"x", "2.jpeg")
        await c.put(b"y", "output_31_0_h3.json")
        assert await c.ls_all("*.jpeg") == ["1.jpeg", "2.jpeg"]
        ok, _ = await c.delete("1.jpeg")
        assert ok and await c.ls("1.jpeg") == []
        assert all(not s.local.has("1.jpeg") for s in nodes.values())
        for s in nodes.values():
            s.ep.stop()

    asyncio.run(main())


def test_rereplication_after_failure(tmp_path):
    async def main():
        net, blobs = LoopbackNetwork(), InProcBlobNetwork()
        names = [f"n{i}" for i in range(6)]
        nodes = _mk(net, blobs, tmp_path, names)
        c = nodes["n0"]
        for i in range(5):
            ok, _ = await c.put(bytes([i]) * 10, f"{i}.jpeg")
            assert ok
        victim = next(n for n in names if n != "n0" and nodes[n].local.all_files())
        net.kill(victim)
        blobs.dead.add(victim)
        for s in nodes.values():
            s.ml.merge({victim: [1, 3, {}]})
        restored = await c.node_failed(victim)
        assert restored >= 1
        for i in range(5):
            hs = c.meta.holders(f"{i}.jpeg")
            assert victim not in hs and len(hs) == 4
            got = await nodes["n2"].get(f"{i}.jpeg")
            assert got[1] == bytes([i]) * 10
        for s in nodes.values():
            s.ep.stop()

    asyncio.run(main())


def test_tcp_blob_server(tmp_path):
    async def main():
        st = LocalFileStore(str(tmp_path / "a"))
        st.put_bytes("f", b"v1")
        st.put_bytes("f", b"v2" * 100000)
        src = BlobSource(st)
        srv = await BlobServer(src).start()
        cli = TcpBlobClient(lambda n: srv.addr)
        assert await cli.fetch("a", {"op": "get", "name": "f", "version": 1}) == [(1, b"v1")]
        allv = await cli.fetch("a", {"op": "get_all", "name": "f"})
        assert [v for v, _ in allv] == [1, 2] and len(allv[1][1]) == 200000
        tok = src.stage(b"pending")
        assert await cli.fetch("a", {"op": "outbox", "token": tok}) == [(0, b"pending")]
        assert await cli.fetch("a", {"op": "get", "name": "missing"}) == []
        srv.close()

    asyncio.run(main())


def test_tcp_blob_server_bad_request_replies_error(tmp_path):
    """A request the source cannot serve (no "name" key, evicted version) gets an
    explicit error reply (ConnectionError at the client, so callers try the next
    holder) and the server keeps serving."""
    async def main():
        st = LocalFileStore(str(tmp_path / "a"))
        st.put_bytes("f", b"v1")
        src = BlobSource(st)
        srv = await BlobServer(src).start()
        cli = TcpBlobClient(lambda n: srv.addr)
        with pytest.raises(ConnectionError):
            await cli.fetch("a", {"op": "get"})  # KeyError in the source
        orig = src.read

        def evicted(req):
            if req.get("op") == "get_all":
                raise FileNotFoundError("version evicted mid get_all")
            return orig(req)
        src.read = evicted
        with pytest.raises(ConnectionError):
            await cli.fetch("a", {"op": "get_all", "name": "f"})
        assert await cli.fetch("a", {"op": "get", "name": "f", "version": 1}) == [(1, b"v1")]
        srv.close()

    asyncio.run(main())


def test_put_many_one_round_trip_per_bundle(tmp_path):
    """put_many: every file on its own replicas (placement as a single PUT), versioned,
    readable; a file already being uploaded is reported failed, not silently dropped;
    replica replies name only the files they stored (no full listings)."""
    async def main():
        net, blobs = LoopbackNetwork(), InProcBlobNetwork()
        names = [f"n{i}" for i in range(6)]
        nodes = _mk(net, blobs, tmp_path, names)
        c, leader = nodes["n4"], nodes["n0"]
        items = [(f"output_31_{b}_rank0.json", f"batch {b}".encode()) for b in range(12)]
        sent = []
        orig = c.ep.request

        async def spy(dest, mtype, payload=None, **kw):
            sent.append(mtype)
            return await orig(dest, mtype, payload, **kw)
        c.ep.request = spy
        ok, failed, err = await c.put_many(items)
        assert sorted(ok) == sorted(n for n, _ in items) and failed == [] and not err
        assert len(sent) == 1  # ONE leader round trip for 12 files
        for n, data in items:
            hs = await c.ls(n)
            assert len(hs) == 4 and set(hs) == set(leader.meta.place(n, names))
            assert await nodes["n5"].get(n) == (1, data)
        ok, failed, _ = await c.put_many(items[:3])      # new versions of existing files
        assert sorted(ok) == sorted(n for n, _ in items[:3])
        assert (await nodes["n1"].get(items[0][0]))[0] == 2
        leader.meta.begin("busy.json", ["n1"])           # an upload in progress is refused, per file
        ok, failed, _ = await c.put_many([("busy.json", b"x"), ("free.json", b"y")])
        assert ok == ["free.json"] and failed == ["busy.json"]
        for s in nodes.values():
            s.ep.stop()

    asyncio.run(main())
