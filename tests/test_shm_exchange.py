"""The service's per-step control exchange over node-local shared memory
(csrc/host/shm_exchange.cpp via parallel/elastic.ShmExchange): all-gather semantics
across processes for thousands of steps, a retry after a timed-out wait does not
publish twice, a member that never publishes (dead) fails the wait through the
failure-detector poll, and the segment is removed at close."""
import multiprocessing as mp
import os
import uuid

import pytest
import torch

from distributed_machine_learning_amd.parallel.elastic import CollectiveFailure, ShmExchange


def _rank(name, world, rank, steps, q):
    ex = ShmExchange(name, world, rank)
    out = torch.zeros((world, 6), dtype=torch.int64)
    bad = 0
    for s in range(1, steps + 1):
        rec = torch.tensor([rank, s, rank * s, 7, 8, 9], dtype=torch.int64)
        ex.exchange(out, rec, poll=lambda: None)
        want = torch.tensor([[r, s, r * s, 7, 8, 9] for r in range(world)], dtype=torch.int64)
        bad += int(not torch.equal(out, want))
    ex.close()
    q.put((rank, bad))


def test_shm_exchange_all_gather_across_processes():
    name = f"/dml_test_{uuid.uuid4().hex[:10]}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(name, 3, r, 3000, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    assert res == {0: 0, 1: 0, 2: 0}
    os.unlink("/dev/shm" + name)


def test_shm_exchange_dead_member_fails_the_wait():
    name = f"/dml_test_{uuid.uuid4().hex[:10]}"
    a = ShmExchange(name, 2, 0)
    polls = []

    def poll():
        polls.append(1)
        if len(polls) >= 3:  # the failure detector confirms rank 1 dead
            raise CollectiveFailure("rank 1 declared dead")
    with pytest.raises(CollectiveFailure):
        a.exchange(torch.zeros((2, 4), dtype=torch.int64), torch.ones(4, dtype=torch.int64), poll, slice_us=1000)
    assert len(polls) == 3
    b = ShmExchange(name, 2, 1)  # a late peer still completes step 1; rank 0 retries without re-publishing
    out_a, out_b = torch.zeros((2, 4), dtype=torch.int64), torch.zeros((2, 4), dtype=torch.int64)
    a.step -= 1  # the caller retries the same step
    b.exchange(out_b, torch.full((4,), 2, dtype=torch.int64), poll=lambda: None)
    a.exchange(out_a, torch.full((4,), 5, dtype=torch.int64), poll=lambda: None)
    assert out_a.tolist() == out_b.tolist() == [[1, 1, 1, 1], [2, 2, 2, 2]]
    a.close()
    b.close(unlink=True)
    assert not os.path.exists("/dev/shm" + name)
    with pytest.raises(CollectiveFailure):  # another geometry under the same name is refused
        ShmExchange(name, 2, 0).close(unlink=False) or ShmExchange(name, 3, 0)
    os.unlink("/dev/shm" + name)
