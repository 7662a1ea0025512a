#!/usr/bin/env python3
"""Start a whole cluster described by a config file on this host (the
reference's README runs 10 copies of main.py by hand, README.md:15-52).

    python tools/launch_cluster.py configs/local10.toml
        [--client-cmd "5 /path/to/testfiles" --client-cmd "submit-job ResNet50 100" ...]
        [--run-for 60] [--log-dir ./logs]

Starts the introducer DNS, then every coordinator/standby/worker entry as its
own process (``serving.main --config F --node NAME``). With ``--client-cmd``
the file's client node runs those commands once everything is up; the
launcher then stops the children it started (after ``--run-for`` seconds, or
on Ctrl-C) and exits with the client's status.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_machine_learning_amd.utils import config as cfgmod  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--client-cmd", action="append", default=[])
    ap.add_argument("--run-for", type=float, default=0.0)
    ap.add_argument("--log-dir", default="./logs")
    ap.add_argument("--startup", type=float, default=2.0, help="seconds to let membership settle")
    a = ap.parse_args()
    c = cfgmod.load(a.config)
    os.makedirs(a.log_dir, exist_ok=True)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    children = []

    def spawn(name, argv):
        log = open(os.path.join(a.log_dir, f"{name}.out"), "w")
        p = subprocess.Popen([sys.executable, "-m"] + argv, stdout=log, stderr=subprocess.STDOUT, env=env)
        children.append(p)
        return p

    if c.introducer:
        host, port = c.introducer.rsplit(":", 1)
        spawn("introducer", ["distributed_machine_learning_amd.cluster.introducer", "-p", port, "-H", host])
        time.sleep(0.5)
    order = c.by_role("coordinator") + c.by_role("standby") + c.by_role("worker")
    for n in order:
        spawn(n.name, ["distributed_machine_learning_amd.serving.main", "--config", a.config, "--node", n.name,
                       "--log", os.path.join(a.log_dir, f"{n.name}.log"), "--exit-after", "1e9", "--cmd", "2"])
        time.sleep(0.1)
    time.sleep(a.startup)
    rc = 0
    try:
        clients = c.by_role("client")
        if a.client_cmd and clients:
            argv = [sys.executable, "-m", "distributed_machine_learning_amd.serving.main", "--config", a.config,
                    "--node", clients[0].name, "--log", os.path.join(a.log_dir, "client.log"), "--exit-after", "0.5"]
            for cmd in a.client_cmd:
                argv += ["--cmd", cmd]
            rc = subprocess.call(argv, env=env)
        if a.run_for:
            time.sleep(a.run_for)
        elif not a.client_cmd:
            print(f"cluster of {len(order)} nodes up (logs in {a.log_dir}); Ctrl-C to stop", flush=True)
            while all(p.poll() is None for p in children):
                time.sleep(1.0)
    except KeyboardInterrupt:
        pass
    finally:
        for p in children:  # only the processes this launcher started
            if p.poll() is None:
                p.terminate()
        for p in children:
            try:
                p.wait(5)
            except subprocess.TimeoutExpired:
                p.kill()
    return rc


if __name__ == "__main__":
    sys.exit(main())
