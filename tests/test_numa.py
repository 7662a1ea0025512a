"""NUMA-local rank placement (utils/numa.py) over a fake sysfs tree: the GPU -> NUMA node
-> cores map the launchers bind each rank to before any GPU call."""
import os

from distributed_machine_learning_amd.utils import numa


def _fake_sysfs(root, gpus_per_node=4, nodes=2, cores=8, drm_numa=True):
    """2 CPU nodes (KFD nodes 0, 1) + 8 GPUs (KFD nodes 2..9): GPU g on NUMA node g // 4."""
    topo = root / "class" / "kfd" / "kfd" / "topology" / "nodes"
    for c in range(nodes):
        d = topo / str(c)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {cores}\nsimd_count 0\n")
        nd = root / "devices" / "system" / "node" / f"node{c}"
        nd.mkdir(parents=True)
        (nd / "cpulist").write_text(f"{c * cores}-{c * cores + cores - 1}\n")
    for g in range(nodes * gpus_per_node):
        d = topo / str(nodes + g)
        d.mkdir(parents=True)
        minor = 128 + g
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count 1024\ndrm_render_minor {minor}\n")
        (d / "io_links" / "0").mkdir(parents=True)
        (d / "io_links" / "0" / "properties").write_text(f"type 2\nnode_from {nodes + g}\nnode_to {g // gpus_per_node}\n")
        dd = root / "class" / "drm" / f"renderD{minor}" / "device"
        dd.mkdir(parents=True)
        (dd / "numa_node").write_text(f"{g // gpus_per_node if drm_numa else -1}\n")
    return str(root)


def test_cpulist_roundtrip():
    assert numa.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert numa.format_cpulist([11, 0, 1, 2, 3, 8, 10]) == "0-3,8,10-11"


def test_gpu_to_numa_node_and_cores(tmp_path):
    sysfs = _fake_sysfs(tmp_path)
    gpus = numa.kfd_gpus(sysfs)
    assert [g["node"] for g in gpus] == list(range(2, 10))
    assert [numa.gpu_numa_node(r, sysfs, env={}) for r in range(8)] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert numa.node_cpus(1, sysfs) == list(range(8, 16))
    # a visibility mask remaps HIP device r to physical GPU mask[r]
    assert numa.gpu_numa_node(0, sysfs, env={"HIP_VISIBLE_DEVICES": "5,2"}) == 1
    assert numa.gpu_numa_node(1, sysfs, env={"ROCR_VISIBLE_DEVICES": "5,2"}) == 0
    assert numa.gpu_numa_node(2, sysfs, env={"HIP_VISIBLE_DEVICES": "5,2"}) is None
    assert numa.gpu_numa_node(8, sysfs, env={}) is None


def test_numa_from_io_link_when_drm_reads_minus_one(tmp_path):
    sysfs = _fake_sysfs(tmp_path, drm_numa=False)
    assert [numa.gpu_numa_node(r, sysfs, env={}) for r in (0, 3, 4, 7)] == [0, 0, 1, 1]


def test_bind_record_intersects_the_allowed_cpuset(tmp_path):
    sysfs = _fake_sysfs(tmp_path)
    allowed = set(os.sched_getaffinity(0))
    rec = numa.bind_local_rank(5, sysfs, env={}, apply=False)
    assert rec["numa"] == 1 and rec["local_rank"] == 5 and rec["bound"] is False
    want = sorted(set(range(8, 16)) & allowed)
    if want:
        assert numa.parse_cpulist(rec["cpus"]) == want
    else:
        assert "cpuset" in rec["reason"]
    assert numa.bind_local_rank(0, sysfs, env={"DML_NUMA_BIND": "0"})["numa"] is None
    assert numa.bind_local_rank(0, str(tmp_path / "none"), env={})["reason"].startswith("no KFD")


def test_bind_applies_the_mask_in_a_child(tmp_path):
    """The mask is really applied (in a child process, so this test process keeps its own)."""
    import multiprocessing as mp

    sysfs = _fake_sysfs(tmp_path, cores=max(1, len(os.sched_getaffinity(0)) // 2))
    q = mp.get_context("fork").Queue()

    def child():
        rec = numa.bind_local_rank(0, sysfs, env={})
        q.put((rec, sorted(os.sched_getaffinity(0))))
    p = mp.get_context("fork").Process(target=child)
    p.start()
    rec, got = q.get(timeout=30)
    p.join(30)
    if rec["bound"]:
        assert got == numa.parse_cpulist(rec["cpus"]) == sorted(set(numa.node_cpus(0, sysfs)) & set(os.sched_getaffinity(0)))
    assert numa.host_threads(share=4, cap=32) >= 2
