"""BASELINE config 1 through the product: the rank launcher with ``--backend cpu``
(HostRankBackend over the fp32 PyTorch executor, serving.inference.CpuBackend), one
rank, batch size 1, the reference's testfiles/ JPEGs loaded into the store by CLI
menu 5, ``submit-job ResNet50 N``, ``get-output``. The merged result has the
reference's output format: download/output_1_127.json maps an image name to
[[[wnid, label, probability] x 5]] (worker.py:1617-1627 writes it). The weights are
random-init (no checkpoints here), so the classes themselves are parity unpinned; the
format, the coverage and the probability ordering are checked, and every row equals
CpuBackend.predict of the same decoded image."""
import asyncio
import json
import os
import socket
import subprocess
import sys

import numpy as np

from distributed_machine_learning_amd.serving.cli import Cli
from distributed_machine_learning_amd.serving.node import Node, NodeConfig

REF_FILES = "/root/reference/testfiles"
REF_OUT = "/root/reference/download/output_1_127.json"
N_IMAGES = 100  # every reference testfile, batch size 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _testfiles(tmp_path, n=N_IMAGES):
    if os.path.isdir(REF_FILES):
        return REF_FILES
    from PIL import Image

    d = tmp_path / "testfiles"
    d.mkdir()
    rng = np.random.default_rng(0)
    for i in range(1, n + 1):
        Image.fromarray(rng.integers(0, 255, (300, 240, 3), dtype=np.uint8)).save(d / f"{i}.jpeg")
    return str(d)


def _ref_format():
    if os.path.exists(REF_OUT):
        with open(REF_OUT) as f:  # JSON text: a safe load
            return json.load(f)
    return {"1.jpeg": [[["n01440764", "tench", 0.5]] * 5]}


def test_rank_launcher_cpu_backend_config1(tmp_path):
    files = _testfiles(tmp_path)
    base = _free_port() - 2
    cmd = [sys.executable, "-m", "distributed_machine_learning_amd.serving.main", "--role", "rank", "--gpus", "1",
           "--backend", "cpu", "--comm", "gloo", "--batch-resnet", "1", "--batch-inception", "1",
           "--base-port", str(base), "--store-dir", str(tmp_path / "sdfs"), "--rdzv", str(tmp_path / "rdzv")]
    env = dict(os.environ, DML_RDZV_DIR=str(tmp_path))
    logf = open(tmp_path / "rank.log", "w")
    proc = subprocess.Popen(cmd, env=env, stdout=logf, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        async def run():
            client = await Node(NodeConfig(role="client", introducer=f"127.0.0.1:{base}",
                                           store_dir=str(tmp_path / "client"), period=0.1, ping_timeout=0.1,
                                           suspect_timeout=1.0)).start()
            for _ in range(240):  # the rank imports torch and builds its control plane first
                await client.join()
                if client.leader() == f"127.0.0.1:{base}":
                    break
                client.fd.stop()
                await asyncio.sleep(0.25)
            assert client.leader() == f"127.0.0.1:{base}"
            cli = Cli(client, testfiles=files, download_dir=str(tmp_path / "download"))
            out = {"load": await cli.run_line(f"5 {files}"),
                   "c3": await cli.run_line("C3 ResNet50 1"),
                   "submit": await cli.run_line(f"submit-job ResNet50 {N_IMAGES}")}
            job = int(out["submit"].split("submitted job ")[1].split()[0])
            out["wait"] = await cli.run_line(f"wait-job {job} 240")
            out["get"] = await cli.run_line(f"get-output {job}")
            # the rank's metrics follow the completions its control loop applies (a relayed
            # transition, not the job table the wait reads): poll C1 a little under load
            for _ in range(40):
                out["c1"] = await cli.run_line("C1")
                try:
                    if json.loads(out["c1"].split("\n[")[0])["ResNet50"]["query_count"] == N_IMAGES:
                        break
                except (ValueError, KeyError):
                    pass
                await asyncio.sleep(0.25)
            await client.stop()
            return job, out
        job, out = asyncio.run(run())
    finally:
        proc.terminate()
        try:
            proc.wait(timeout=60)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, 9)
            proc.wait()
        logf.close()
        log = open(tmp_path / "rank.log").read()
    assert "finished" in out["wait"], (out, log[-3000:])
    assert json.loads(out["c1"].split("\n[")[0])["ResNet50"]["query_count"] == N_IMAGES
    text = open(tmp_path / "download" / f"final_{job}.json").read()
    final = json.loads(text)
    assert len(final) == N_IMAGES
    assert text == json.dumps(final, indent=4)          # the reference's indent-4 layout
    # the per-batch files the rank PUT into its store: reference-formatted, one per batch
    import glob

    stored = [f for f in glob.glob(str(tmp_path / "sdfs" / "**" / f"output_{job}_*"), recursive=True)]
    assert stored
    from distributed_machine_learning_amd.serving.output import dumps

    one = open(stored[0]).read()
    assert one == dumps(json.loads(one))
    ref = _ref_format()
    rv = next(iter(ref.values()))
    for name, v in final.items():
        assert name.endswith(".jpeg")
        # same nesting as the reference file: one list holding 5 [wnid, label, prob] triples
        assert isinstance(v, list) and len(v) == len(rv) == 1 and len(v[0]) == len(rv[0]) == 5
        for trip, rt in zip(v[0], rv[0]):
            assert [type(x) for x in trip] == [type(x) for x in rt]
            assert trip[0].startswith("n") and len(trip[0]) == 9
        probs = [t[2] for t in v[0]]
        assert probs == sorted(probs, reverse=True) and 0.0 <= probs[-1] and probs[0] <= 1.0

    # every row is the CPU executor's top-5 of the same decoded image
    from distributed_machine_learning_amd.serving.inference import CpuBackend
    from distributed_machine_learning_amd.utils.labels import load_class_index

    be = CpuBackend()
    names = sorted(final)
    blobs = [open(os.path.join(files, n), "rb").read() for n in names]
    idx, p = be.predict("ResNet50", be.decode_batch("ResNet50", blobs))
    wnids = [w for w, _ in load_class_index()]
    for i, n in enumerate(names):
        assert [t[0] for t in final[n][0]] == [wnids[j] for j in idx[i]], n
        np.testing.assert_allclose([t[2] for t in final[n][0]], p[i], rtol=1e-4, atol=1e-6)
