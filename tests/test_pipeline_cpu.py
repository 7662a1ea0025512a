"""parallel/pipeline.py's issue order on CPU (gloo, world 2): the real ServingPipeline
with a fake engine and image store. With the lagged gather (world > 1 default) the
result gather of batch k goes out after forward k+1 and the host consumes batch k after
the gather of k+1 was issued; every rank issues its collectives (dispatch broadcasts,
result gathers) in the same order, and rank 0 receives each batch's rows from the right
step and rank."""
import json
import os
import socket
import time

import numpy as np
import torch
import torch.multiprocessing as mp

B = 4


class _Engine:
    device = "cpu"
    src_slots = 2
    batch = B

    def __init__(self, rank, delay):
        self.rank, self.delay = rank, delay
        self.srcs = [torch.zeros(B, dtype=torch.int64) for _ in range(2)]
        self.results = [torch.zeros((2, B, 5), dtype=torch.int32) for _ in range(2)]

    def run(self, stream, use_graph=True, slot=0):
        time.sleep(self.delay)  # a slow rank: skew the gathers see
        r = self.results[slot]
        r.zero_()
        r[0, :, 0] = self.srcs[slot].to(torch.int32)
        r[0, :, 1] = self.rank


class _Store:
    def h2d(self, dst, start, count, stream):
        dst[:count] = torch.arange(start, start + count)


def _rank(rank, world, port, out, lag, lookahead):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from distributed_machine_learning_amd.parallel.dataplane import DataPlane
    from distributed_machine_learning_amd.parallel.pipeline import ServingPipeline

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dp = DataPlane(torch.device("cpu"), result_shape=(2, B, 5))
    got = {}

    def on_results(rec):
        got[rec.step] = [t[0, :, :2].tolist() for t in rec.results]
    pipe = ServingPipeline(_Engine(rank, 0.002 * rank), _Store(), dp, use_graph=False, on_results=on_results,
                           lookahead=lookahead, gather_lag=lag)

    def table(k):
        return np.array([[31, k, 0, (k * world + r) * B, B, 0] for r in range(world)], np.int64)
    steps = 9
    pipe.run(steps, table)
    with open(os.path.join(out, f"pipe_{rank}.json"), "w") as f:
        json.dump({"order": pipe.order, "got": got, "lag": pipe.gather_lag}, f)
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(tmp_path, lag, lookahead):
    world = 2
    ctx = mp.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, str(tmp_path), lag, lookahead)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    assert [p.exitcode for p in ps] == [0, 0]
    return [json.load(open(tmp_path / f"pipe_{r}.json")) for r in range(world)]


def _check(res, lag):
    steps = 9
    r0, r1 = res
    # the collectives go out in the same order on every rank
    coll = [[tuple(x) for x in r["order"] if x[0] in ("dispatch", "gather")] for r in res]
    assert coll[0] == coll[1]
    order = [tuple(x) for x in r0["order"]]
    pos = {op: i for i, op in enumerate(order)}
    for k in range(steps):
        assert pos[("forward", k)] < pos[("gather", k)] < pos[("finish", k)]
        if lag and k + 1 < steps:
            assert pos[("forward", k + 1)] < pos[("gather", k)]    # gather k after forward k+1
            assert pos[("gather", k + 1)] < pos[("finish", k)]     # consumed after the next gather went out
        if not lag and k + 1 < steps:
            assert pos[("gather", k)] < pos[("forward", k + 1)]
    # rank 0 got every batch's rows from the right step and rank
    for k in range(steps):
        rows = r0["got"][str(k)]
        for r in range(2):
            assert rows[r] == [[(k * 2 + r) * B + i, r] for i in range(B)], (k, r, rows[r])


def test_pipeline_lagged_gather_order_gloo(tmp_path):
    res = _run(tmp_path, None, 2)
    assert res[0]["lag"] == 1   # world > 1: the lagged gather is the default
    _check(res, 1)


def test_pipeline_inline_gather_order_gloo(tmp_path):
    _check(_run(tmp_path, 0, 1), 0)
