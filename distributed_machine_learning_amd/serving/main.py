"""Node entry point (reference main.py:15-77: ``python3 main.py --hostname=H
--port=P [-t]``; logging to debug.log + stdout; SIGINT/SIGTERM stop the node).

  python -m distributed_machine_learning_amd.serving.main --hostname 127.0.0.1 --port 8001 \
      --role coordinator --introducer 127.0.0.1:8888 [--backend gpu|cpu|fake] [-t] \
      [--cmd "5 /path/to/testfiles" --cmd "submit-job ResNet50 100" ...]

  python -m distributed_machine_learning_amd.serving.main --config configs/local10.toml --node H3

  python -m distributed_machine_learning_amd.serving.main --role rank --gpus 8     # the MI355X service
      (serving/rank_main.py: one rank process per GPU; the CLI connects with --role client)

With ``--config`` the node takes its role, address, backend and every cluster
setting from the file's entry for ``--node`` (utils/config.py); flags given
explicitly on the command line still override the file. ``--trace out.json``
writes a Chrome trace of the node's job / batch lifecycle at exit.

With no ``--cmd`` the node runs the interactive stdin menu (cli.py); with
``--cmd`` it executes the commands in order and keeps serving until
``--exit-after`` seconds (or forever).
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import signal
import sys

from .cli import MENU, Cli
from .node import Node, NodeConfig
from ..cluster.tasks import spawn


def parse(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(description="distributed inference node")
    ap.add_argument("-H", "--hostname", default="127.0.0.1")
    ap.add_argument("-p", "--port", type=int, default=None)
    ap.add_argument("--config", default="", help="cluster config file (TOML/JSON), utils/config.py")
    ap.add_argument("--node", default="", help="this node's name / host:port / index in --config")
    ap.add_argument("--journal", default=None, help="coordinator job journal (restart recovery)")
    ap.add_argument("--trace", default="", help="write a Chrome trace of this node at exit")
    ap.add_argument("-t", "--testing", action="store_true", help="3%% send drop + bps/false-positive meters")
    ap.add_argument("--role", default="worker", choices=["coordinator", "standby", "worker", "client", "rank"])
    ap.add_argument("--introducer", default="127.0.0.1:8888")
    ap.add_argument("--seed-node", action="append", default=[])
    ap.add_argument("--store-dir", default="./sdfs")
    ap.add_argument("--download-dir", default="./download")
    ap.add_argument("--testfiles", default="")
    ap.add_argument("--backend", default="cpu", choices=["gpu", "cpu", "fake", "store"])
    ap.add_argument("--gpu", type=int, default=0)
    ap.add_argument("--period", type=float, default=0.5)
    ap.add_argument("--ping-timeout", type=float, default=0.25)
    ap.add_argument("--suspect-timeout", type=float, default=2.0)
    ap.add_argument("--cleanup", type=float, default=10.0)
    ap.add_argument("--batch-size", type=int, default=10)
    ap.add_argument("--cmd", action="append", default=[])
    ap.add_argument("--exit-after", type=float, default=0.0)
    ap.add_argument("--log", default="debug.log")
    from .rank_main import add_args

    add_args(ap)
    a = ap.parse_args(argv)
    # flags given on the command line (even when equal to their defaults: ``--backend cpu``
    # on a rank overrides the rank's own default, its GPU)
    argv_l = sys.argv[1:] if argv is None else list(argv)
    given = {t.split("=", 1)[0] for t in argv_l if t.startswith("--")}
    a.explicit = {k for k, v in vars(a).items()
                  if v != ap.get_default(k) or "--" + k.replace("_", "-") in given}
    if a.role == "rank":
        return a
    if a.port is None and not (a.config and a.node):
        ap.error("--port is required (or --config with --node)")
    return a


def node_config(a: argparse.Namespace) -> NodeConfig:
    """Build this node's NodeConfig from the flags, or from --config/--node
    with explicitly given flags layered on top."""
    kw = {}
    if a.backend == "gpu":
        kw = {"device": f"cuda:{a.gpu}"}
    if not a.config:
        return NodeConfig(host=a.hostname, port=a.port, role=a.role, introducer=a.introducer or None,
                          seeds=a.seed_node, store_dir=a.store_dir, out_dir=None, backend=a.backend, backend_kw=kw,
                          testing=a.testing, period=a.period, ping_timeout=a.ping_timeout,
                          suspect_timeout=a.suspect_timeout, cleanup_time=a.cleanup,
                          batch_sizes={"ResNet50": a.batch_size, "InceptionV3": a.batch_size}, journal=a.journal)
    from ..utils import config as _config

    cluster = _config.load(a.config)
    ex = a.explicit
    ov = {"period": a.period if "period" in ex else None,
          "ping_timeout": a.ping_timeout if "ping_timeout" in ex else None,
          "suspect_timeout": a.suspect_timeout if "suspect_timeout" in ex else None,
          "cleanup_time": a.cleanup if "cleanup" in ex else None,
          "store_dir": a.store_dir if "store_dir" in ex else None,
          "testing": True if "testing" in ex else None,
          "journal": a.journal if "journal" in ex else None,
          "introducer": a.introducer if "introducer" in ex else None}
    if "batch_size" in ex:
        ov["batch_sizes"] = {"ResNet50": a.batch_size, "InceptionV3": a.batch_size}
    cfg = cluster.node_config(a.node or str(a.port), **ov)
    for flag, attr in (("hostname", "host"), ("port", "port"), ("role", "role"), ("backend", "backend")):
        if flag in ex:
            setattr(cfg, attr, getattr(a, flag))
    if "backend" in ex or "gpu" in ex:
        cfg.backend_kw = kw
    if "seed_node" in ex:
        cfg.seeds = a.seed_node
    if not a.testfiles and cluster.testfiles:
        a.testfiles = cluster.testfiles
    if "download_dir" not in ex:
        a.download_dir = cluster.download_dir
    return cfg


async def amain(a: argparse.Namespace) -> int:
    cfg = node_config(a)
    if a.trace:
        from ..utils import trace as _trace

        tr = _trace.set_tracer(_trace.Tracer(process_name=f"node {cfg.host}:{cfg.port} ({cfg.role})"))
    node = await Node(cfg).start()
    await node.join()
    cli = Cli(node, testfiles=a.testfiles, download_dir=a.download_dir)
    loop = asyncio.get_running_loop()
    stop = asyncio.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, stop.set)
        except NotImplementedError:  # pragma: no cover
            pass
    if a.cmd:
        for line in a.cmd:
            print(await cli.run_line(line), flush=True)
        if a.exit_after:
            try:
                await asyncio.wait_for(stop.wait(), a.exit_after)
            except asyncio.TimeoutError:
                pass
            await node.stop()
            if a.trace:
                tr.export_chrome(a.trace)
            return 0
    else:
        print(MENU, flush=True)
        q: asyncio.Queue = asyncio.Queue()
        loop.add_reader(sys.stdin, lambda: q.put_nowait(sys.stdin.readline()))

        async def reader():
            while True:
                line = await q.get()
                if not line:
                    stop.set()
                    return
                print(await cli.run_line(line), flush=True)

        spawn(reader(), loop)
    await stop.wait()
    await node.stop()
    if a.trace:
        tr.export_chrome(a.trace)
    return 0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse(argv)
    if a.role == "rank":
        from . import rank_main

        if a.rank < 0:
            return rank_main.launch(a, argv)
        return rank_main.rank_main(a)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s",
                        handlers=[logging.FileHandler(a.log), logging.StreamHandler(sys.stderr)])
    return asyncio.run(amain(a))


if __name__ == "__main__":
    sys.exit(main())
