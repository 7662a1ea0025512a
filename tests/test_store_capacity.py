"""Output-store capacity at the 8-GPU batch rate (VERDICT r4 "next round" 3), CPU only.

gloo world 8 of the shipped serving product (parallel/service_bench.run via
tools/store_capacity.py): the collective service, the per-rank control plane, the replicated
store with R = 4, every output rendered by the native renderer (~170 KB of indent-4 JSON per
ResNet50 b256 batch) and durable on its 4 replicas before its batch is reported, each rank's
GPU replaced by a backend that completes 600 batches/s (PacedRankBackend): what is measured is
the host side alone. Asserted: every batch's output is in the store exactly once (one name per
(job, batch), no duplicates, none failed) and the sustained rate. The requirement is 8 x 360
batches/s (8 GPUs x ResNet50 b256) with a 25 % margin; a GPU node gives each rank cores of its
own, and the rate assertion applies where the host has them (>= 64 CPUs, e.g. a gpurun box: tools/store_capacity.py
is its harness, results in profiles/). On this container's 8 shared cores the 8 rank processes
(3 busy threads each) are CPU-bound near 8 x 80 and the test asserts a floor that catches a
collapse of the path (the r4 leader fan-out ran 8 x 17 here)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.serial
def test_output_store_capacity_world8(tmp_path):
    import store_capacity

    world, rate = 8, 600.0   # offered: 8 x 600 batches/s, above the 1.25 x 8 x 360 asserted below
    rec = store_capacity.measure(world, rate, batches_per_rank=200, tmp=str(tmp_path))
    cap, out = rec["capacity"], rec["outputs"]
    nb = rec["batches"]["ResNet50"]
    print("store capacity", json.dumps(cap))
    assert rec["jobs_done"] and nb == world * 200
    # a batch re-run after a rebuild writes a new version of the same name: >= nb files written,
    # exactly nb distinct outputs listed
    assert out["files_stored"] >= nb and out["failed"] == 0, (out, rec.get("rebuilds"))
    assert out["in_store"] == nb and out["distinct_batches_in_store"] == nb and out["listing_duplicates"] == 0
    assert cap["bytes_per_output"] > 120_000                      # real-size outputs
    # a 25 % margin over the 8-GPU rate where the host has the cores (a gpurun
    # box sustained 4,229 batches/s offered 8 x 600, profiles/r6_final/capacity_w8_rate600.json)
    need = 1.25 * world * 360
    if (os.cpu_count() or 1) >= 64:
        assert cap["batches_per_s"] >= need, cap
    else:
        assert cap["batches_per_s"] >= world * 40, cap
