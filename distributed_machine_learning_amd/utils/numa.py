"""NUMA-local placement of the one-process-per-GPU ranks (VERDICT r4 "next round" 4).

On an 8 x MI355X node each GPU hangs off one CPU socket. A rank's host side — the
pinned H2D arenas it streams every batch from (about 14 GB/s per GPU in the bench
pipeline), its JPEG decode pool and its output writer — belongs on the cores of that
socket: a pinned buffer is placed by first touch, so a rank whose threads run on the
far socket pulls every image across the inter-socket link before it reaches PCIe.

The reference ran one process per VM (``main.py:15-27``), so placement never arose
there; here it is intrinsic to "one process per GPU on one node".

Everything is read from sysfs, never through a GPU API (the launchers bind before any
HIP call, and children inherit the mask):

* GPUs are the KFD topology nodes with ``simd_count > 0``
  (``/sys/class/kfd/kfd/topology/nodes/<n>/properties``), in KFD node order — the order
  ROCr enumerates its GPU agents in, i.e. HIP device order when no visibility mask is set
  (``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``, numeric
  lists, remap it);
* a GPU's NUMA node is ``/sys/class/drm/renderD<drm_render_minor>/device/numa_node``, or,
  where that reads -1, the CPU node its first KFD io_link points to (``node_to``);
* the node's cores are ``/sys/devices/system/node/node<k>/cpulist``, intersected with the
  process's allowed set (a container cpuset); an empty intersection binds nothing.

``DML_NUMA_BIND=0`` turns the binding off (A/B).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def _props(text: str) -> Dict[str, int]:
    out = {}
    for line in text.splitlines():
        parts = line.split()
        if len(parts) == 2:
            try:
                out[parts[0]] = int(parts[1])
            except ValueError:
                pass
    return out


def parse_cpulist(s: str) -> List[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]"""
    cpus: List[int] = []
    for part in s.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            cpus.extend(range(int(a), int(b) + 1))
        else:
            cpus.append(int(part))
    return cpus


def format_cpulist(cpus) -> str:
    """[0, 1, 2, 3, 8, 10, 11] -> '0-3,8,10-11'"""
    cpus = sorted(set(cpus))
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def kfd_gpus(sysfs: str = "/sys") -> List[dict]:
    """The GPU nodes of the KFD topology in node order: [{"node", "render_minor", "numa"}]."""
    root = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    try:
        nodes = sorted((int(d) for d in os.listdir(root) if d.isdigit()))
    except OSError:
        return []
    gpus = []
    for n in nodes:
        p = _props(_read(os.path.join(root, str(n), "properties")) or "")
        if p.get("simd_count", 0) <= 0:
            continue  # a CPU node
        minor = p.get("drm_render_minor", -1)
        numa = -1
        txt = _read(os.path.join(sysfs, "class", "drm", f"renderD{minor}", "device", "numa_node")) if minor >= 0 else None
        if txt is not None:
            try:
                numa = int(txt.strip())
            except ValueError:
                numa = -1
        if numa < 0:  # the CPU node of the GPU's first io_link
            lp = _props(_read(os.path.join(root, str(n), "io_links", "0", "properties")) or "")
            to = lp.get("node_to", -1)
            cp = _props(_read(os.path.join(root, str(to), "properties")) or "") if to >= 0 else {}
            if to >= 0 and cp.get("simd_count", 0) == 0 and cp.get("cpu_cores_count", 0) > 0:
                numa = to
        gpus.append({"node": n, "render_minor": minor, "numa": numa})
    return gpus


def _visible(env) -> Optional[List[int]]:
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(k)
        if v is None or v.strip() == "":
            continue
        try:
            return [int(x) for x in v.split(",") if x.strip()]
        except ValueError:
            return None  # UUID forms: no mapping from sysfs
    return None


def gpu_numa_node(local_rank: int, sysfs: str = "/sys", env=None) -> Optional[int]:
    """NUMA node of HIP device ``local_rank`` (None: unknown)."""
    env = os.environ if env is None else env
    gpus = kfd_gpus(sysfs)
    vis = _visible(env)
    idx = local_rank
    if vis is not None:
        if local_rank >= len(vis):
            return None
        idx = vis[local_rank]
    if idx < 0 or idx >= len(gpus):
        return None
    n = gpus[idx]["numa"]
    return n if n >= 0 else None


def node_cpus(node: int, sysfs: str = "/sys") -> List[int]:
    txt = _read(os.path.join(sysfs, "devices", "system", "node", f"node{node}", "cpulist"))
    return parse_cpulist(txt) if txt else []


def bind_local_rank(local_rank: int, sysfs: str = "/sys", env=None, apply: bool = True) -> dict:
    """Bind this process (and the threads it starts later) to the cores of GPU
    ``local_rank``'s NUMA node. Returns the record the bench prints:
    {"local_rank", "numa", "cpus", "bound"}."""
    env = os.environ if env is None else env
    rec = {"local_rank": local_rank, "numa": None, "cpus": None, "bound": False}
    if env.get("DML_NUMA_BIND", "1") == "0":
        rec["reason"] = "DML_NUMA_BIND=0"
        return rec
    node = gpu_numa_node(local_rank, sysfs, env)
    if node is None:
        rec["reason"] = "no KFD / NUMA topology for this GPU"
        return rec
    rec["numa"] = node
    try:
        allowed = set(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = set(range(os.cpu_count() or 1))
    cpus = sorted(set(node_cpus(node, sysfs)) & allowed)
    if not cpus:
        rec["reason"] = "the node's cores are outside this process's cpuset"
        rec["cpus"] = format_cpulist(sorted(allowed))
        return rec
    rec["cpus"] = format_cpulist(cpus)
    if apply:
        try:
            os.sched_setaffinity(0, cpus)
            rec["bound"] = True
        except OSError as e:
            rec["reason"] = f"sched_setaffinity: {e}"
    return rec


def host_threads(share: int = 1, cap: int = 32) -> int:
    """Worker threads for a rank's host pools (JPEG decode): this rank's share of the cores
    it is bound to (``share`` = the ranks bound to the same cores), at least 2, at most ``cap``."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 8
    return max(2, min(cap, n // max(1, share)))


def ranks_sharing(local_rank: int, local_world: int, sysfs: str = "/sys", env=None) -> int:
    """How many of the node's ``local_world`` ranks sit on ``local_rank``'s NUMA node
    (1 when the topology is unknown): the share a rank's host pools are sized by."""
    node = gpu_numa_node(local_rank, sysfs, env)
    if node is None:
        return 1
    return max(1, sum(1 for r in range(local_world) if gpu_numa_node(r, sysfs, env) == node))
