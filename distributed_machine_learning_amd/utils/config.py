"""Cluster configuration files (TOML or JSON) + command-line overrides.

Reference: module-level constants in config.py (the static 10-VM cluster
H1..H10, config.py:54-63; FD constants M / PING_TIMEOOUT / PING_DURATION /
CLEANUP_TIME, config.py:4-10; paths, config.py:17-19; introducer address,
config.py:25-26) and roles hard-coded by hostname (H1 leader, H2 standby,
H3..H10 workers: worker.py:52, election.py:27). Here one file describes the
whole cluster; every node process picks its own entry by name and the role
comes from the file, not from the hostname:

    [cluster]
    introducer = "127.0.0.1:8888"
    period = 0.5            # FD probe period (s); reference 12 s
    batch_size = 10
    [[nodes]]
    name = "H1"
    port = 8001
    role = "coordinator"
    [[nodes]]
    name = "H3"
    port = 8003
    role = "worker"
    backend = "gpu"
    gpu = 0

Precedence: built-in defaults < ``[cluster]`` < the node's own table <
explicit command-line flags.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

ROLES = ("coordinator", "standby", "worker", "client")


@dataclass
class NodeSpec:
    name: str
    port: int
    host: str = "127.0.0.1"
    role: str = "worker"
    backend: str = "cpu"
    gpu: int = 0
    extra: Dict[str, Any] = field(default_factory=dict)  # per-node overrides of cluster keys

    @property
    def addr(self) -> str:
        return f"{self.host}:{self.port}"


@dataclass
class ClusterConfig:
    nodes: List[NodeSpec] = field(default_factory=list)
    introducer: Optional[str] = "127.0.0.1:8888"
    period: float = 0.5
    ping_timeout: float = 0.25
    suspect_timeout: float = 2.0
    cleanup_time: float = 10.0
    replication: int = 4
    batch_size: int = 10
    batch_sizes: Dict[str, int] = field(default_factory=dict)
    store_dir: str = "./sdfs"
    download_dir: str = "./download"
    testfiles: str = ""
    journal: Optional[str] = None
    testing: bool = False
    drop_rate: float = 0.03

    def node(self, key) -> NodeSpec:
        """Look a node up by name, ``host:port``, port or index."""
        for i, n in enumerate(self.nodes):
            if key in (n.name, n.addr, str(n.port), n.port, i, str(i)):
                return n
        raise KeyError(f"no node {key!r} in the cluster config")

    def by_role(self, role: str) -> List[NodeSpec]:
        return [n for n in self.nodes if n.role == role]

    def node_config(self, key, **overrides):
        """The NodeConfig of one node (serving/node.py)."""
        from ..serving.node import NodeConfig

        spec = self.node(key)
        merged = {k: getattr(self, k) for k in _CLUSTER_KEYS}
        merged.update(spec.extra)
        merged.update({k: v for k, v in overrides.items() if v is not None})
        bs = dict(merged.get("batch_sizes") or {})
        for m in ("ResNet50", "InceptionV3"):
            bs.setdefault(m, int(merged["batch_size"]))
        kw = {"device": f"cuda:{spec.gpu}"} if spec.backend == "gpu" else {}
        seeds = [n.addr for n in self.nodes if n.role == "coordinator" and n.name != spec.name]
        return NodeConfig(host=spec.host, port=spec.port, role=spec.role, introducer=merged["introducer"],
                          seeds=seeds, store_dir=merged["store_dir"], backend=spec.backend, backend_kw=kw,
                          testing=bool(merged["testing"]), drop_rate=float(merged["drop_rate"]),
                          period=float(merged["period"]), ping_timeout=float(merged["ping_timeout"]),
                          suspect_timeout=float(merged["suspect_timeout"]),
                          cleanup_time=float(merged["cleanup_time"]), replication=int(merged["replication"]),
                          batch_sizes=bs, journal=merged.get("journal") if spec.role == "coordinator" else None)


_CLUSTER_KEYS = tuple(f.name for f in dataclasses.fields(ClusterConfig) if f.name != "nodes")
_NODE_KEYS = tuple(f.name for f in dataclasses.fields(NodeSpec) if f.name != "extra")


def load_file(path: str) -> Dict[str, Any]:
    with open(path, "rb") as f:
        raw = f.read()
    if path.endswith((".toml", ".tml")):
        try:
            import tomllib as _toml  # py >= 3.11
        except ImportError:  # pragma: no cover - py3.10 here
            import tomli as _toml
        return _toml.loads(raw.decode())
    return json.loads(raw)


def from_dict(d: Dict[str, Any]) -> ClusterConfig:
    c = dict(d.get("cluster", {}))
    unknown = set(c) - set(_CLUSTER_KEYS)
    if unknown:
        raise ValueError(f"unknown [cluster] keys: {sorted(unknown)}")
    nodes = []
    for i, nd in enumerate(d.get("nodes", [])):
        nd = dict(nd)
        base = {k: nd.pop(k) for k in list(nd) if k in _NODE_KEYS}
        if "name" not in base:
            base["name"] = f"H{i + 1}"
        if base.get("role", "worker") not in ROLES:
            raise ValueError(f"node {base['name']}: role must be one of {ROLES}")
        bad = set(nd) - set(_CLUSTER_KEYS)
        if bad:
            raise ValueError(f"node {base['name']}: unknown keys {sorted(bad)}")
        nodes.append(NodeSpec(**base, extra=nd))
    names = [n.name for n in nodes]
    if len(set(names)) != len(names):
        raise ValueError("duplicate node names")
    addrs = [n.addr for n in nodes]
    if len(set(addrs)) != len(addrs):
        raise ValueError("duplicate node addresses")
    return ClusterConfig(nodes=nodes, **c)


def load(path: str) -> ClusterConfig:
    return from_dict(load_file(path))


def to_dict(cfg: ClusterConfig) -> Dict[str, Any]:
    c = {k: getattr(cfg, k) for k in _CLUSTER_KEYS}
    nodes = []
    for n in cfg.nodes:
        d = {k: getattr(n, k) for k in _NODE_KEYS}
        d.update(n.extra)
        nodes.append(d)
    return {"cluster": c, "nodes": nodes}


def reference_layout(base_port: int = 8001, gpu_workers: int = 0, host: str = "127.0.0.1") -> ClusterConfig:
    """The reference's 10-node shape (H1 coordinator, H2 standby, H3..H10
    workers; config.py:54-63, worker.py:52) on one host; the first
    ``gpu_workers`` workers get GPUs 0..gpu_workers-1."""
    nodes = [NodeSpec("H1", base_port, host, "coordinator"), NodeSpec("H2", base_port + 1, host, "standby")]
    for i in range(8):
        gpu = i < gpu_workers
        nodes.append(NodeSpec(f"H{i + 3}", base_port + 2 + i, host, "worker", "gpu" if gpu else "cpu", i if gpu else 0))
    return ClusterConfig(nodes=nodes)


def save(cfg: ClusterConfig, path: str) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    with open(path, "w") as f:
        json.dump(to_dict(cfg), f, indent=2)
    return path
