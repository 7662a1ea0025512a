"""The serving product on the GPU (VERDICT r2, next-round item 1 "done means"):
``serving.main --role rank --gpus 1`` with the default GPU backend (native
engines of both models + HBM image stores fed by the replicated store), driven
by the reference CLI from a client node: load the testfiles, submit a job, wait,
merge the outputs the rank wrote and PUT into the store; then re-PUT one image
and run a second job (version pinning). Every output row must equal the
engine run directly on the decoded bytes of the version the job pinned.
"""
import asyncio
import json

import numpy as np
import pytest
import torch

from test_rank_service import REPO, _free_port, _jpegs


pytestmark = pytest.mark.gpu


def _launch_logged(tmp_path, world):
    """The launcher with its (and its ranks') output in a file: a GPU rank
    logs more than a pipe nobody drains would hold."""
    import os
    import subprocess
    import sys
    import time

    base = _free_port()
    while base + world + 2 > 64000:
        base = _free_port()
    logf = open(tmp_path / "launcher.log", "w")
    cmd = [sys.executable, "-m", "distributed_machine_learning_amd.serving.main", "--role", "rank", "--gpus",
           str(world), "--backend", "gpu", "--base-port", str(base), "--store-dir", str(tmp_path / "sdfs"),
           "--batch-resnet", "8", "--batch-inception", "8", "--replication", "1", "--arena-images", "256"]
    p = subprocess.Popen(cmd, cwd=REPO, stdout=logf, stderr=subprocess.STDOUT, text=True, start_new_session=True)
    for _ in range(600):
        txt = open(tmp_path / "launcher.log").read()
        if "rank-service:" in txt or p.poll() is not None:
            break
        time.sleep(0.1)
    assert "rank-service:" in txt, txt
    return p, base


def _stop_logged(p, tmp_path):
    import os
    import signal
    import subprocess

    try:
        os.killpg(p.pid, signal.SIGTERM)
        p.wait(timeout=120)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.wait()
    return p.returncode, open(tmp_path / "launcher.log").read()[-6000:]


async def _client_slow(introducer, tmp_path):
    """Like test_rank_service._client, but waits for a rank that is still
    building its engines (the rank answers only after its control plane starts)."""
    from distributed_machine_learning_amd.serving.node import Node, NodeConfig

    client = await Node(NodeConfig(role="client", introducer=introducer, store_dir=str(tmp_path / "client"),
                                   period=0.1, ping_timeout=0.1, suspect_timeout=1.0)).start()
    for _ in range(600):
        await client.join()
        if client.leader() is not None:
            break
        client.fd.stop()
        await asyncio.sleep(0.25)
    return client


def _engine_rows(blobs, names):
    """top-5 ids / probs of ResNet50 on the decoded blobs, 4 images per pass
    (the SplitEngine halves of the rank's batch-8 engine)."""
    from distributed_machine_learning_amd.models import build_model
    from distributed_machine_learning_amd.models.engine import Engine
    from distributed_machine_learning_amd.serving.inference import load_image

    g, w = build_model("ResNet50", seed=0)
    e = Engine(g, w, batch=4)
    out = {}
    for b0 in range(0, len(names), 4):
        chunk = names[b0:b0 + 4]
        pad = torch.zeros((4, 224, 224, 3), dtype=torch.uint8)
        for i, n in enumerate(chunk):
            pad[i] = torch.from_numpy(load_image(blobs[n], (224, 224)))
        e.infer(pad.cuda())
        torch.cuda.synchronize()
        r = e.result.cpu()
        for i, n in enumerate(chunk):
            out[n] = (r[0, i].tolist(), r[1, i].view(torch.float32).numpy())
    return out


@pytest.mark.timeout(900)
@pytest.mark.parametrize("force_gather", [False, True])
def test_gpu_rank_launcher_cli_roundtrip(tmp_path, monkeypatch, force_gather):
    """force_gather: the result rows reach the coordinator through a one-rank RCCL gather on
    the result group (DML_COLLECT_FORCE_GATHER: the collective path of get-output on one GPU)."""
    import os

    from PIL import Image

    if force_gather:
        monkeypatch.setenv("DML_COLLECT_FORCE_GATHER", "1")
    files = _jpegs(str(tmp_path / "testfiles"))
    p, base = _launch_logged(tmp_path, 1)
    try:
        async def run():
            from distributed_machine_learning_amd.serving.cli import Cli

            client = await _client_slow(f"127.0.0.1:{base}", tmp_path)
            cli = Cli(client, testfiles=files, download_dir=str(tmp_path / "dl"))
            out = {"load": await cli.run_line(f"5 {files}"),
                   "submit": await cli.run_line("submit-job ResNet50 12"),
                   "wait": await cli.run_line("wait-job 31 300"),
                   "get": await cli.run_line("get-output 31")}
            out["fast"] = client.last_output_fast   # rendered at the coordinator from gathered rows
            out["slow"] = await client.merge_output_files(31, str(tmp_path / "slow_31.json"))
            v2 = str(tmp_path / "3v2.jpeg")
            Image.fromarray(np.full((40, 30, 3), 200, np.uint8)).save(v2)
            out["put"] = await cli.run_line(f"put {v2} 3.jpeg")
            out["submit2"] = await cli.run_line("submit-job ResNet50 12")
            out["wait2"] = await cli.run_line("wait-job 32 300")
            out["get2"] = await cli.run_line("get-output 32")
            out["c1"] = await cli.run_line("C1")
            await client.stop()
            return out, open(v2, "rb").read()
        out, v2bytes = asyncio.run(run())
    finally:
        rc, log = _stop_logged(p, tmp_path)
    assert "loaded 12/12" in out["load"], (out, log)
    assert "finished" in out["wait"] and "finished" in out["wait2"], (out, log)
    assert out["fast"] is True, (out, log)
    assert open(out["slow"], "rb").read() == open(tmp_path / "dl" / "final_31.json", "rb").read()
    f1 = json.load(open(tmp_path / "dl" / "final_31.json"))
    f2 = json.load(open(tmp_path / "dl" / "final_32.json"))
    assert sorted(f1) == sorted(f2) == sorted(f"{i}.jpeg" for i in range(1, 13))
    assert f1["3.jpeg"] != f2["3.jpeg"]
    from distributed_machine_learning_amd.utils.labels import load_class_index

    cls = {wnid: i for i, (wnid, _) in enumerate(load_class_index())}
    blobs = {n: open(os.path.join(files, n), "rb").read() for n in f1}
    for doc, bl in ((f1, blobs), (f2, dict(blobs, **{"3.jpeg": v2bytes}))):
        ref = _engine_rows(bl, sorted(doc))
        for n, ent in doc.items():
            ids, pr = ref[n]
            assert [cls[e[0]] for e in ent[0]] == ids, n
            assert np.allclose([e[2] for e in ent[0]], pr, rtol=0, atol=0), n
    c1 = json.loads(out["c1"].split("\n[")[0])
    assert c1["ResNet50"]["query_count"] == 24
    assert rc == 0, log
