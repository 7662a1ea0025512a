"""Auxiliary subsystems: Chrome-trace tracing, cluster config files
with command-line overrides, and the coordinator's job journal (restart
recovery)."""
import asyncio
import json
import os
import textwrap

import pytest

from distributed_machine_learning_amd.cluster.frames import Frame, MsgType
from distributed_machine_learning_amd.serving.coordinator import Coordinator
from distributed_machine_learning_amd.serving.journal import JobJournal
from distributed_machine_learning_amd.utils import config as cfgmod
from distributed_machine_learning_amd.utils import trace


# ------------------------------------------------------------------ tracing --
def test_tracer_host_spans_async_and_chrome_export(tmp_path):
    t = trace.Tracer(process_name="t")
    with t.span("outer", step=1):
        with t.span("inner"):
            pass
    t.instant("tick", k=3)
    t.begin_async("batch", "31:1", worker="w0")
    t.end_async("batch", "31:1", outcome="done")
    t.counter("queue", ResNet50=4, InceptionV3=2)
    t.add_gpu_ops([("conv1", 0.5), ("pool", 0.25)], lane="ops")
    path = t.export_chrome(str(tmp_path / "trace.json"))
    doc = json.load(open(path))
    evs = doc["traceEvents"]
    names = [e["name"] for e in evs]
    for n in ("outer", "inner", "tick", "batch", "queue", "conv1", "pool", "process_name", "thread_name"):
        assert n in names
    outer = next(e for e in evs if e["name"] == "outer")
    inner = next(e for e in evs if e["name"] == "inner")
    assert outer["ph"] == "X" and outer["args"] == {"step": 1}
    assert outer["ts"] <= inner["ts"] and inner["ts"] + inner["dur"] <= outer["ts"] + outer["dur"] + 1e-3
    assert [e["ph"] for e in evs if e["name"] == "batch"] == ["b", "e"]
    conv, pool = (next(e for e in evs if e["name"] == n) for n in ("conv1", "pool"))
    assert conv["dur"] == pytest.approx(500.0) and pool["ts"] == pytest.approx(conv["ts"] + 500.0)
    s = t.summary()
    assert s["conv1"]["count"] == 1 and s["conv1"]["total_ms"] == pytest.approx(0.5)


def test_disabled_tracer_records_nothing():
    t = trace.Tracer(enabled=False)
    with t.span("x"):
        pass
    with t.gpu_span("y", stream=None):
        pass
    t.instant("z")
    t.begin_async("a", 1)
    assert [e for e in t.events() if e["ph"] != "M"] == []


def test_merge_rank_traces(tmp_path):
    paths = []
    for r in range(2):
        t = trace.Tracer(process_name=f"rank {r}", pid=r)
        with t.span("step"):
            pass
        paths.append(t.export_chrome(str(tmp_path / f"r{r}.json")))
    out = trace.merge_chrome(paths, str(tmp_path / "all.json"))
    evs = json.load(open(out))["traceEvents"]
    assert {e["pid"] for e in evs if e["name"] == "step"} == {0, 1}


@pytest.mark.gpu
def test_gpu_span_resolves_on_device():
    import torch

    t = trace.Tracer()
    s = torch.cuda.Stream()
    x = torch.randn(2048, 2048, device="cuda")
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), t.gpu_span("matmul", s, lane="compute"):
        for _ in range(4):
            x = x @ x.T / 2048
    ev = [e for e in t.events() if e["name"] == "matmul"]
    assert len(ev) == 1 and ev[0]["dur"] > 0 and ev[0]["cat"] == "gpu"


# ------------------------------------------------------------------- config --
TOML = textwrap.dedent("""
    [cluster]
    introducer = "127.0.0.1:9888"
    period = 0.2
    batch_size = 16
    journal = "/tmp/j.jsonl"

    [[nodes]]
    name = "H1"
    port = 9001
    role = "coordinator"

    [[nodes]]
    name = "H2"
    port = 9002
    role = "standby"

    [[nodes]]
    name = "H3"
    port = 9003
    role = "worker"
    backend = "gpu"
    gpu = 3
    period = 0.1
""")


def test_config_toml_precedence(tmp_path):
    p = tmp_path / "c.toml"
    p.write_text(TOML)
    c = cfgmod.load(str(p))
    assert [n.name for n in c.nodes] == ["H1", "H2", "H3"] and c.by_role("worker")[0].gpu == 3
    w = c.node_config("H3")
    assert w.role == "worker" and w.port == 9003 and w.backend_kw == {"device": "cuda:3"}
    assert w.period == 0.1  # node table beats [cluster]
    assert w.batch_sizes == {"ResNet50": 16, "InceptionV3": 16} and w.introducer == "127.0.0.1:9888"
    assert w.journal is None and c.node_config("H1").journal == "/tmp/j.jsonl"  # coordinator only
    assert c.node_config("127.0.0.1:9002").role == "standby" and c.node_config(9001).role == "coordinator"
    assert w.seeds == ["127.0.0.1:9001"]
    # command-line flags beat the file
    from distributed_machine_learning_amd.serving.main import node_config, parse

    a = parse(["--config", str(p), "--node", "H3", "--period", "0.05", "--batch-size", "64"])
    nc = node_config(a)
    assert nc.period == 0.05 and nc.batch_sizes["ResNet50"] == 64 and nc.ping_timeout == 0.25
    a = parse(["--config", str(p), "--node", "H3"])
    assert node_config(a).period == 0.1


def test_config_json_roundtrip_and_errors(tmp_path):
    ref = cfgmod.reference_layout(gpu_workers=8)
    assert [n.role for n in ref.nodes] == ["coordinator", "standby"] + ["worker"] * 8
    assert [n.gpu for n in ref.by_role("worker")] == list(range(8))
    p = cfgmod.save(ref, str(tmp_path / "ref.json"))
    back = cfgmod.load(p)
    assert cfgmod.to_dict(back) == cfgmod.to_dict(ref)
    with pytest.raises(ValueError):
        cfgmod.from_dict({"cluster": {"bogus": 1}})
    with pytest.raises(ValueError):
        cfgmod.from_dict({"nodes": [{"name": "a", "port": 1, "role": "king"}]})
    with pytest.raises(ValueError):
        cfgmod.from_dict({"nodes": [{"name": "a", "port": 1}, {"name": "a", "port": 2}]})
    with pytest.raises(KeyError):
        ref.node("H99")


def test_shipped_configs_parse():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = os.path.join(root, "configs")
    files = [f for f in os.listdir(d) if f.endswith((".toml", ".json"))]
    assert files
    for f in files:
        c = cfgmod.load(os.path.join(d, f))
        assert c.by_role("coordinator") and c.by_role("worker")
        for n in c.nodes:
            c.node_config(n.name)


# ------------------------------------------------------------------ journal --
class _Ep:
    def __init__(self):
        self.sent = []

    def on(self, *a):
        pass

    async def send(self, dest, mtype, payload=None, seq=0):
        self.sent.append((dest, mtype, payload))

    async def reply(self, fr, mtype, payload=None):
        pass

    async def request(self, dest, mtype, payload=None, timeout=2.0, retries=0):
        return Frame(MsgType.ACK, dest, {})


class _Member:
    meta = {"role": "worker"}


class _Ml:
    def __init__(self, workers):
        self.workers = workers

    def alive(self, include_self=True):
        return list(self.workers)

    def get(self, n):
        return _Member() if n in self.workers else None

    def is_alive(self, n):
        return n in self.workers


def _coord(journal, workers=("w1", "w2")):
    images = [f"{i}.jpeg" for i in range(10)]
    return Coordinator(_Ep(), _Ml(workers), list_images=lambda pat: images, locate=lambda img: {"w1": [1]},
                       batch_sizes={"ResNet50": 4, "InceptionV3": 4}, journal=journal)


def test_journal_recovers_coordinator_state(tmp_path):
    path = str(tmp_path / "jobs.jsonl")

    async def first():
        c = _coord(JobJournal(path))
        job = await c.submit("ResNet50", 40, "client")          # 10 batches
        assert job.job_id == 31
        assert await c.schedule() == 2                          # two in flight
        inflight = sorted(k for _, k, _ in c.running.values())
        worker = next(w for w, (_, k, _) in c.running.items() if k == inflight[0])
        await c._on_worker_ack(Frame(MsgType.WORKER_TASK_REQUEST_ACK, worker,
                                     {"jobid": 31, "batchid": inflight[0][1], "model": "ResNet50",
                                      "image_count": 4, "service_time": 0.01}))
        await c._on_set_batch_size(Frame(MsgType.SET_BATCH_SIZE, "client", {"model": "InceptionV3",
                                                                             "batch_size": 7}))
        c.journal.close()
        return inflight, {k for _, k, _ in c.running.values()}

    inflight, still_running = asyncio.run(first())
    assert len(still_running) == 2  # the ACK freed a worker and a new batch was dispatched

    async def second():
        c = _coord(JobJournal(path))                             # "restart" on the same journal
        assert c.recovered > 0
        j = c.jobs.jobs[31]
        assert j.batches_done == 1 and j.batches_total == 10
        q = [b.key for b in c.jobs.queues["ResNet50"]]
        assert len(q) == 9 and set(q[:2]) == still_running      # in-flight went to the front
        assert inflight[0] not in q
        assert c.jobs.batch_sizes["InceptionV3"] == 7 and not c.running
        job2 = await c.submit("InceptionV3", 7, "client")
        assert job2.job_id == 32
        c.journal.close()

    asyncio.run(second())
    # compaction left one snapshot line + the new submit
    ops = [e["op"] for e in JobJournal(path).entries()]
    assert ops[0] == "snapshot" and ops[1:] == ["submit"]


def test_journal_skips_torn_line(tmp_path):
    p = tmp_path / "j.jsonl"
    j = JobJournal(str(p))
    j.append("batch_size", model="ResNet50", batch_size=3)
    j.close()
    with open(p, "a") as f:
        f.write('{"op": "subm')  # crash mid-write
    assert [e["op"] for e in JobJournal(str(p)).entries()] == ["batch_size"]


# ---------------------------------------------------- multi-process launcher --
def _free_ports(n):
    import socket

    socks, ports = [], []
    for _ in range(n):
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def test_launch_cluster_from_config(tmp_path):
    """tools/launch_cluster.py: introducer + coordinator + 2 workers as separate
    processes over real UDP/TCP, driven by a client node from the same file."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pi, pc, pw1, pw2, pcl = _free_ports(5)
    cfg = {"cluster": {"introducer": f"127.0.0.1:{pi}", "period": 0.2, "store_dir": str(tmp_path / "sdfs"),
                       "journal": str(tmp_path / "journal.jsonl"), "batch_size": 4},
           "nodes": [{"name": "H1", "port": pc, "role": "coordinator"},
                     {"name": "H3", "port": pw1, "backend": "fake"},
                     {"name": "H4", "port": pw2, "backend": "fake"},
                     {"name": "cli", "port": pcl, "role": "client"}]}
    path = tmp_path / "c.json"
    path.write_text(json.dumps(cfg))
    imgs = tmp_path / "imgs"
    imgs.mkdir()
    for i in range(6):
        (imgs / f"{i}.jpeg").write_bytes(b"x" * (100 + i))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "launch_cluster.py"), str(path),
                        "--log-dir", str(tmp_path / "logs"), "--startup", "1.5",
                        "--client-cmd", f"5 {imgs}", "--client-cmd", "submit-job ResNet50 12",
                        "--client-cmd", "C5"], capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "loaded 6/6 files" in r.stdout and "submitted job 31" in r.stdout
    ops = [e["op"] for e in JobJournal(str(tmp_path / "journal.jsonl")).entries()]
    assert ops[0] == "submit" and "dispatch" in ops


# ------------------------------------------------- asyncio debug-mode run --
def test_cluster_job_clean_under_asyncio_debug(tmp_path, caplog):
    """The in-process cluster (coordinator + standby + workers + client) serves
    a job with asyncio debug mode on: no coroutine is left un-awaited and no
    task dies with an exception nobody retrieved (the reference's fire-and-
    forget create_task pattern, worker.py:1188, loses both silently)."""
    import gc
    import logging
    import warnings

    from test_serving import _cluster, _load_images, _stop

    async def main():
        asyncio.get_running_loop().slow_callback_duration = 5.0  # only correctness, not timing
        net, blobs, nodes = await _cluster(tmp_path, n_workers=3)
        cli = nodes["cli"]
        await _load_images(cli, 6)
        jid = await cli.submit_job("ResNet50", 20)
        assert await cli.wait_job(jid, timeout=20)
        net.kill("w1")  # a failure mid-run exercises the requeue / FD paths too
        jid2 = await cli.submit_job("InceptionV3", 12)
        assert await cli.wait_job(jid2, timeout=30)
        await _stop(nodes)

    with warnings.catch_warnings(record=True) as rec, caplog.at_level(logging.ERROR, logger="asyncio"):
        warnings.simplefilter("always")
        asyncio.run(main(), debug=True)
        gc.collect()
    never_awaited = [str(w.message) for w in rec if "was never awaited" in str(w.message)]
    assert not never_awaited, never_awaited
    bad = [r.getMessage() for r in caplog.records if "never retrieved" in r.getMessage()]
    assert not bad, bad
