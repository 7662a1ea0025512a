"""BASELINE config 1 ("plumbing"): ResNet50, batch size 1, a single CPU worker,
on the reference's testfiles JPEGs — driven through the CLI command surface,
over real UDP sockets + TCP blob servers on 127.0.0.1. Also covers every
store/menu command. The reference images are read from /root/reference
(read-only); if absent, synthetic JPEGs of the same shape are generated."""
import asyncio
import io
import json
import os

import numpy as np
import pytest

from distributed_machine_learning_amd.serving.cli import Cli
from distributed_machine_learning_amd.serving.node import Node, NodeConfig

REF_FILES = "/root/reference/testfiles"


def _testfiles(tmp_path, n=6):
    if os.path.isdir(REF_FILES):
        return REF_FILES
    from PIL import Image

    d = tmp_path / "testfiles"
    d.mkdir()
    rng = np.random.default_rng(0)
    for i in range(1, n + 1):
        Image.fromarray(rng.integers(0, 255, (300, 240, 3), dtype=np.uint8)).save(d / f"{i}.jpeg")
    return str(d)


def test_plumbing_resnet50_bs1_cpu_worker(tmp_path):
    files = _testfiles(tmp_path)

    async def main():
        base = dict(store_dir=str(tmp_path / "sdfs"), period=0.1, ping_timeout=0.1, suspect_timeout=1.0,
                    cleanup_time=5.0, replication=2, store_timeout=5.0)
        coord = await Node(NodeConfig(role="coordinator", **base)).start()
        await coord.join()
        worker = await Node(NodeConfig(role="worker", backend="cpu", seeds=[coord.name], **base)).start()
        await worker.join()
        client = await Node(NodeConfig(role="client", seeds=[coord.name], **base)).start()
        await client.join()
        await asyncio.sleep(0.5)
        cli = Cli(client, testfiles=files, download_dir=str(tmp_path / "download"))
        # load only a handful of the 100 reference JPEGs to keep the CPU test short
        sub = tmp_path / "sub"
        sub.mkdir()
        for f in sorted(os.listdir(files))[:5]:
            (sub / f).write_bytes(open(os.path.join(files, f), "rb").read())
        out = await cli.run_line(f"5 {sub}")
        assert "loaded 5/5" in out, out
        assert "set to 1" in await cli.run_line("C3 ResNet50 1")
        out = await cli.run_line("submit-job ResNet50 5")
        assert "submitted job 31" in out, out
        assert "finished" in await cli.run_line("wait-job 31 240")
        out = await cli.run_line("get-output 31")
        assert "final_31.json" in out
        final = json.load(open(tmp_path / "download" / "final_31.json"))
        assert len(final) == 5
        for v in final.values():
            assert len(v) == 1 and len(v[0]) == 5
            ps = [e[2] for e in v[0]]
            assert ps == sorted(ps, reverse=True) and 0 < sum(ps) <= 1.0001
        c1 = json.loads((await cli.run_line("C1")).split("\n[")[0])
        assert c1["ResNet50"]["query_count"] == 5
        c2 = json.loads((await cli.run_line("C2")).split("\n[")[0])
        assert c2["ResNet50"]["batches"] == 5
        assert "{}" in await cli.run_line("C5")
        # store commands
        p = tmp_path / "local.txt"
        p.write_text("v1")
        assert "ok" in await cli.run_line(f"put {p} notes.txt")
        p.write_text("v2")
        assert "ok" in await cli.run_line(f"put {p} notes.txt")
        assert "notes.txt" in await cli.run_line("ls-all *.txt")
        assert "got notes.txt v2" in await cli.run_line(f"get notes.txt {tmp_path / 'back.txt'}")
        assert (tmp_path / "back.txt").read_text() == "v2"
        await cli.run_line(f"get-versions notes.txt 2 {tmp_path / 'vers.txt'}")
        assert b"version 1" in (tmp_path / "vers.txt").read_bytes()
        assert "ok" in await cli.run_line("delete notes.txt")
        assert "notes.txt: []" in await cli.run_line("ls notes.txt")
        for opt in ("1", "2", "6", "7", "8", "9", "10", "store", "help"):
            assert "took" in await cli.run_line(opt)
        out = await cli.run_line("predict-locally ResNet50 99 2")
        assert "predicted 2 images" in out
        for n in (client, worker, coord):
            await n.stop()

    asyncio.run(main())
