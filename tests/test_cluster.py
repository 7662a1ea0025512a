"""Control plane: wire format, SWIM membership, failure detector, election,
introducer — all on the in-process loopback network with a fake clock where
timing matters (SURVEY §4 'do better' items 1-2)."""
import asyncio

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from distributed_machine_learning_amd.cluster.election import Election
from distributed_machine_learning_amd.cluster.failure_detector import FailureDetector
from distributed_machine_learning_amd.cluster.frames import (Frame, FrameError, MsgType, Reassembler, decode, encode)
from distributed_machine_learning_amd.cluster.introducer import IntroducerService, fetch_leader, update_leader
from distributed_machine_learning_amd.cluster.membership import MembershipList, Status
from distributed_machine_learning_amd.cluster.transport import Endpoint, LoopbackNetwork, UdpTransport


# ------------------------------------------------------------------ frames --
def test_frame_roundtrip_small():
    f = Frame(MsgType.WORKER_TASK_REQUEST, "10.0.0.1:8001", {"jobid": 31, "images": ["a", "b"]}, seq=7, flags=1)
    dgs = encode(f)
    assert len(dgs) == 1
    g = decode(dgs[0])
    assert (g.type, g.sender, g.payload, g.seq, g.is_reply) == (f.type, f.sender, f.payload, 7, True)


def test_large_payload_fragments_and_reassembles():
    # the reference silently dropped anything over 32 KiB (~122 images per task)
    imgs = {f"{i}.jpeg": {"h3:8003": [1, 2, 3]} for i in range(5000)}
    f = Frame(MsgType.WORKER_TASK_REQUEST, "n:1", {"images": imgs})
    dgs = encode(f)
    assert len(dgs) > 10 and all(len(d) <= 1400 for d in dgs)
    r = Reassembler()
    out = None
    for d in reversed(dgs):  # any arrival order
        out = r.feed(d) or out
    assert out is not None and out.payload["images"] == imgs and r.pending() == 0


def test_bad_datagrams_rejected():
    with pytest.raises(FrameError):
        decode(b"xx")
    with pytest.raises(FrameError):
        decode(b"ZZ" + b"\0" * 40)


@given(st.dictionaries(st.text(max_size=8), st.integers() | st.text(max_size=20), max_size=30),
       st.sampled_from(list(MsgType)))
@settings(max_examples=50, deadline=None)
def test_frame_property_roundtrip(payload, mtype):
    f = Frame(mtype, "h:1", payload, seq=3)
    r = Reassembler()
    out = None
    for d in encode(f, mtu_payload=64):
        out = r.feed(d) or out
    assert out.payload == payload and out.type == mtype


# -------------------------------------------------------------- membership --
class Clock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t


def test_membership_precedence_and_refute():
    c = Clock()
    a = MembershipList("a", clock=c, incarnation=1)
    a.merge({"b": [5, 1, {}]})
    assert a.is_alive("b")
    a.merge({"b": [5, 2, {}]})          # same incarnation, SUSPECT beats ALIVE
    assert a.get("b").status == Status.SUSPECT
    a.merge({"b": [5, 1, {}]})          # stale ALIVE ignored
    assert a.get("b").status == Status.SUSPECT
    a.merge({"b": [6, 1, {}]})          # refutation (higher incarnation)
    assert a.get("b").status == Status.ALIVE
    # a hears itself suspected -> bumps its incarnation
    a.merge({"a": [1, 2, {}]})
    assert a.me.incarnation == 2 and a.me.status == Status.ALIVE


def test_suspect_confirm_purge_callbacks():
    c = Clock()
    events = []
    a = MembershipList("a", clock=c, suspect_timeout=3, cleanup_time=10, incarnation=1)
    a.on_fail.append(lambda n: events.append(("fail", n)))
    a.on_purge.append(lambda n: events.append(("purge", n)))
    a.merge({"b": [1, 1, {}], "c": [1, 1, {}]})
    a.suspect("b")
    c.t = 2.9
    a.tick()
    assert a.get("b").status == Status.SUSPECT
    c.t = 3.0
    a.tick()
    assert a.get("b").status == Status.DEAD and events == [("fail", "b")]
    c.t = 13.0
    a.tick()
    assert a.get("b") is None and events[-1] == ("purge", "b")
    assert a.alive() == ["a", "c"]


def test_false_positive_counter():
    a = MembershipList("a", clock=Clock(), incarnation=1)
    a.merge({"b": [1, 1, {}]})
    a.suspect("b")
    a.mark_alive("b", 1)
    assert a.false_positives == 1 and a.false_positive_rate() == 1.0


def test_ring_targets_reference_offsets():
    names = [f"n{i}" for i in range(10)]
    a = MembershipList("n0", clock=Clock(), incarnation=1)
    a.merge({n: [1, 1, {}] for n in names[1:]})
    assert a.ring_targets() == ["n1", "n9", "n4"]  # [i+1, i-1, i+4] like config.py:67-89
    a.merge({"n1": [1, 3, {}]})                   # dead neighbour is skipped
    assert a.ring_targets() == ["n2", "n9", "n5"]


@given(st.lists(st.tuples(st.sampled_from(["b", "c", "d"]), st.integers(0, 5), st.sampled_from([1, 2, 3])),
                max_size=40))
@settings(max_examples=100, deadline=None)
def test_merge_is_order_independent_for_final_state(updates):
    """Applying the same gossip in any order converges to the same (inc, status)."""
    def run(seq):
        m = MembershipList("a", clock=Clock(), incarnation=100)
        for n, inc, s in seq:
            m.merge({n: [inc, s, {}]})
        return {n: (x.incarnation, x.status) for n, x in m.members.items() if n != "a"}

    assert run(updates) == run(list(reversed(updates)))


# ------------------------------------------------------ detector + election --
async def _cluster(n, net, period=0.05, eligible=("n0", "n1"), standby="n1"):
    nodes = {}
    for i in range(n):
        name = f"n{i}"
        ep = Endpoint(net.transport(name))
        meta = {"role": "standby" if name == standby else ("coordinator" if name == "n0" else "worker"),
                "eligible": name in eligible}
        ml = MembershipList(name, suspect_timeout=0.2, cleanup_time=1.0, meta=meta, incarnation=1)
        fd = FailureDetector(ep, ml, period=period, ping_timeout=0.05)
        el = Election(ep, ml, timeout=0.1)
        ml.on_fail.append(el.leader_failed)
        ep.start()
        nodes[name] = (ep, ml, fd, el)
    for name, (ep, ml, fd, el) in nodes.items():
        if name != "n0":
            assert await fd.join("n0")
    for name, (ep, ml, fd, el) in nodes.items():
        el.set_leader("n0")
        fd.start()
    return nodes


def _stop(nodes):
    for ep, ml, fd, el in nodes.values():
        fd.stop()
        ep.stop()


def test_detector_converges_and_detects_kill():
    async def main():
        net = LoopbackNetwork()
        nodes = await _cluster(6, net)
        await asyncio.sleep(0.4)
        for ep, ml, fd, el in nodes.values():
            assert len(ml.alive()) == 6
        net.kill("n4")
        await asyncio.sleep(1.0)
        for name, (ep, ml, fd, el) in nodes.items():
            if name != "n4":
                assert "n4" not in ml.alive(), (name, ml.table())
        _stop(nodes)

    asyncio.run(main())


def test_no_false_removal_under_packet_loss():
    """Indirect probes keep a lossy (10 %) cluster intact."""
    async def main():
        net = LoopbackNetwork(seed=3)
        nodes = await _cluster(6, net)
        net.set_drop_rate(0.10)
        await asyncio.sleep(1.5)
        for ep, ml, fd, el in nodes.values():
            assert len(ml.alive()) == 6, ml.table()
        _stop(nodes)

    asyncio.run(main())


def test_leader_failure_elects_standby():
    async def main():
        net = LoopbackNetwork()
        nodes = await _cluster(5, net)
        await asyncio.sleep(0.3)
        net.kill("n0")
        await asyncio.sleep(1.5)
        for name, (ep, ml, fd, el) in nodes.items():
            if name != "n0":
                assert el.leader == "n1", (name, el.leader)
        _stop(nodes)

    asyncio.run(main())


def test_election_without_standby_picks_highest_eligible():
    """Reference bug: nobody could win if H2 was dead (election.py:27)."""
    async def main():
        net = LoopbackNetwork()
        nodes = await _cluster(5, net, eligible=("n0", "n1", "n2", "n3"), standby=None)
        await asyncio.sleep(0.3)
        net.kill("n0")
        await asyncio.sleep(1.5)
        leaders = {el.leader for name, (ep, ml, fd, el) in nodes.items() if name != "n0"}
        assert leaders == {"n3"}
        _stop(nodes)

    asyncio.run(main())


def test_introducer_fetch_update():
    async def main():
        net = LoopbackNetwork()
        dns = Endpoint(net.transport("dns"))
        svc = IntroducerService(dns)
        a = Endpoint(net.transport("a"))
        dns.start()
        a.start()
        assert await fetch_leader(a, "dns") == "a"   # first asker becomes introducer
        assert await update_leader(a, "dns", "b")
        assert await fetch_leader(a, "dns") == "b" and svc.updates == 1
        dns.stop()
        a.stop()

    asyncio.run(main())


def test_udp_transport_request_reply():
    async def main():
        t1 = await UdpTransport("127.0.0.1", 0).start()
        t2 = await UdpTransport("127.0.0.1", 0).start()
        e1, e2 = Endpoint(t1), Endpoint(t2)

        async def echo(fr):
            await e2.reply(fr, MsgType.ACK, {"echo": fr.payload})

        e2.on(MsgType.PING, echo)
        e1.start()
        e2.start()
        big = {"x": "y" * 50000}
        r = await e1.request(t2.name, MsgType.PING, big, timeout=2)
        assert r is not None and r.payload["echo"] == big
        assert t1.bytes_sent > 50000
        e1.stop()
        e2.stop()

    asyncio.run(main())


def test_ring_targets_empty_after_leave():
    """leave() marks self LEFT; a probe round afterwards must not raise (it used to
    call ring.index(self) on an alive-list without self and kill the FD task)."""
    ml = MembershipList("a:1")
    ml.merge({"b:1": [0, 1, {}], "c:1": [0, 1, {}]})
    assert ml.ring_targets()
    ml.leave()
    assert ml.ring_targets() == []
