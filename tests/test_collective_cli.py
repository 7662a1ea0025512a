"""One system: the reference's CLI drives the RCCL collective service (here
gloo, world 3, fake backend) — menu 5 loads the reference testfiles into the
store, C3 sets the batch size, ``submit-job ResNet50 100`` is served by the
ranks from store images (decoded once per rank), ``get-output`` merges the
output files the coordinator PUT into the store — and the merged result equals
the host-mode cluster's for the same commands (reference worker.py:176-245,
1617-1627, 1973-1997)."""
import asyncio
import json
import os
import socket
import time

import numpy as np
import torch.multiprocessing as mp

from distributed_machine_learning_amd.serving.cli import Cli
from distributed_machine_learning_amd.serving.node import Node, NodeConfig

REF_FILES = "/root/reference/testfiles"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _testfiles(tmp_path, n=100):
    if os.path.isdir(REF_FILES):
        return REF_FILES
    from PIL import Image

    d = tmp_path / "testfiles"
    d.mkdir()
    rng = np.random.default_rng(0)
    for i in range(1, n + 1):
        Image.fromarray(rng.integers(0, 255, (300, 240, 3), dtype=np.uint8)).save(d / f"{i}.jpeg")
    return str(d)


def _rank_main(grank, world, rdzv, base, out):
    import logging
    import threading

    logging.basicConfig(level=logging.WARNING)
    from distributed_machine_learning_amd.parallel.elastic import ElasticGroup
    from distributed_machine_learning_amd.parallel.service import (CollectiveService, FakeRankBackend, OutputWriter,
                                                                   RankControl, ReplicatedCoordinator)

    eg = ElasticGroup(grank, world, store_path=rdzv, backend="gloo", timeout_s=60)
    ctl = RankControl(grank, world, base, store_dir=os.path.join(out, "sdfs"), replication=2,
                      on_dead=eg.dead.add).start()
    coord = ReplicatedCoordinator({"ResNet50": 16, "InceptionV3": 16}, cap=16, host_tag="mi355x")
    writer = OutputWriter(None, put_many_async=ctl.store_put_many_async, host_tag="mi355x")
    svc = CollectiveService(eg, FakeRankBackend(cap=16, loader=ctl.store_loader), coord, control=ctl,
                            writer=writer, idle_sleep=0.005)

    def stopper():
        while not os.path.exists(os.path.join(out, "STOP")):
            time.sleep(0.05)
        svc.stop()
    threading.Thread(target=stopper, daemon=True).start()
    svc.serve()
    eg.barrier()
    ctl.stop()
    eg.close()


async def _commands(cli, files):
    out = {}
    out["load"] = await cli.run_line(f"5 {files}")
    out["c3"] = await cli.run_line("C3 ResNet50 10")
    out["submit"] = await cli.run_line("submit-job ResNet50 100")
    out["wait"] = await cli.run_line("wait-job 31 120")
    out["get"] = await cli.run_line("get-output 31")
    out["c1"] = await cli.run_line("C1")
    out["c2"] = await cli.run_line("C2")
    out["c5"] = await cli.run_line("C5")
    return out


def test_cli_drives_collective_service_and_matches_host_mode(tmp_path):
    files = _testfiles(tmp_path)
    world, base = 3, _free_port() - 4
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_rank_main, args=(r, world, str(tmp_path / "rdzv"), base, str(tmp_path)))
          for r in range(world)]
    for p in ps:
        p.start()
    try:
        async def collective():
            want = f"127.0.0.1:{base + world - 1}"
            client = await Node(NodeConfig(role="client", introducer=f"127.0.0.1:{base}",
                                           store_dir=str(tmp_path / "client"), period=0.1, ping_timeout=0.1,
                                           suspect_timeout=1.0)).start()
            for _ in range(60):  # any rank answers FETCH_INTRODUCER once its election has settled
                await client.join()
                if client.leader() == want:
                    break
                client.fd.stop()
                await asyncio.sleep(0.25)
            assert client.leader() == want
            cli = Cli(client, testfiles=files, download_dir=str(tmp_path / "dl_collective"))
            out = await _commands(cli, files)
            await client.stop()
            return out
        out = asyncio.run(collective())
    finally:
        (tmp_path / "STOP").write_text("1")
        for p in ps:
            p.join(60)
        for p in ps:
            if p.is_alive():
                p.kill()
    assert "loaded 100/100" in out["load"], out["load"]
    assert "set to 10" in out["c3"], out["c3"]
    assert "submitted job 31" in out["submit"], out["submit"]
    assert "finished" in out["wait"], out["wait"]
    assert "final_31.json" in out["get"], out["get"]
    c1 = json.loads(out["c1"].split("\n[")[0])
    assert c1["ResNet50"]["query_count"] == 100
    c2 = json.loads(out["c2"].split("\n[")[0])
    assert c2["ResNet50"]["batches"] == 10
    assert json.loads(out["c5"].split("\nrecent batches")[0].split("\n[")[0]) == {}
    assert "(ResNet50) ran on rank" in out["c5"]          # C5 history: which rank ran each batch
    final_c = json.load(open(tmp_path / "dl_collective" / "final_31.json"))
    assert len(final_c) == 100

    # the same commands against the host-mode cluster (coordinator + 2 fake-GPU workers)
    async def host_mode():
        kw = dict(store_dir=str(tmp_path / "host_sdfs"), period=0.1, ping_timeout=0.1, suspect_timeout=1.0,
                  cleanup_time=5.0, replication=2, store_timeout=5.0)
        coord = await Node(NodeConfig(role="coordinator", **kw)).start()
        await coord.join()
        workers = []
        for _ in range(2):
            w = await Node(NodeConfig(role="worker", backend="fake", seeds=[coord.name], **kw)).start()
            await w.join()
            workers.append(w)
        client = await Node(NodeConfig(role="client", seeds=[coord.name], **kw)).start()
        await client.join()
        await asyncio.sleep(0.5)
        cli = Cli(client, testfiles=files, download_dir=str(tmp_path / "dl_host"))
        out = await _commands(cli, files)
        for n in (client, *workers, coord):
            await n.stop()
        return out
    out_h = asyncio.run(host_mode())
    assert "finished" in out_h["wait"], out_h
    final_h = json.load(open(tmp_path / "dl_host" / "final_31.json"))
    assert final_c == final_h
