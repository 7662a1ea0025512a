"""Elastic collective serving on CPU (gloo, world 3): concurrent ResNet50 +
InceptionV3 jobs scheduled fair-share over the ranks, then an injected worker
kill mid-job -> SWIM detects it -> rank 0 requeues the step's batches ->
survivors re-form the communicator (epoch 1) -> every job still completes.
(BASELINE configs 4/5 in miniature; the GPU version swaps gloo for RCCL and the
fake backend for the native engines.)"""
import json
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(grank, world, store_port, swim_base, out, kill_rank, kill_step):
    import logging

    logging.basicConfig(level=logging.WARNING)
    from distributed_machine_learning_amd.parallel.elastic import ElasticGroup
    from distributed_machine_learning_amd.parallel.fd_thread import RankFailureDetector
    from distributed_machine_learning_amd.parallel.service import (CollectiveCoordinator, CollectiveService,
                                                                   FakeRankBackend)

    eg = ElasticGroup(grank, world, port=store_port, backend="gloo", timeout_s=30)
    fd = RankFailureDetector(grank, world, swim_base, on_dead=eg.dead.add).start()
    coord = None
    if grank == 0:
        coord = CollectiveCoordinator({"ResNet50": 8, "InceptionV3": 8}, {"ResNet50": 64, "InceptionV3": 64},
                                      out_dir=os.path.join(out, "outputs"), host_tag="test")
        jobs = [coord.submit("ResNet50", 96), coord.submit("InceptionV3", 96)]
    svc = CollectiveService(eg, FakeRankBackend(max_batch=8, delay_per_image=0.002), coord,
                            kill_rank=kill_rank, kill_at_step=kill_step)
    steps = svc.serve(max_steps=500)
    if grank == 0:
        coord.flush()
        res = {"steps": steps, "rebuilds": svc.rebuilds, "epoch": eg.epoch, "members": eg.members,
               "done": [coord.jobs.jobs[j].done for j in jobs], "requeued": coord.requeued,
               "c1": coord.metrics.c1(), "c2": coord.metrics.c2(),
               "outputs": len(os.listdir(os.path.join(out, "outputs")))}
        with open(os.path.join(out, "result.json"), "w") as f:
            json.dump(res, f)
    fd.stop()
    eg.close()


def _run(tmp_path, kill_rank=-1, kill_step=-1, world=3):
    ctx = mp.get_context("spawn")
    sp, swim = _free_port(), _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, sp, swim, str(tmp_path), kill_rank, kill_step))
          for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(180)
    for p in ps:
        if p.is_alive():
            p.kill()
    with open(tmp_path / "result.json") as f:
        return json.load(f), [p.exitcode for p in ps]


def test_concurrent_models_fair_share(tmp_path):
    res, codes = _run(tmp_path)
    assert codes == [0, 0, 0]
    assert res["done"] == [True, True] and res["rebuilds"] == 0
    assert res["c1"]["ResNet50"]["query_count"] == 96 and res["c1"]["InceptionV3"]["query_count"] == 96
    assert res["outputs"] == 24  # 12 + 12 batches of 8


def test_worker_kill_mid_job_recovers(tmp_path):
    res, codes = _run(tmp_path, kill_rank=2, kill_step=3)
    assert codes[2] == 17 and codes[0] == 0 and codes[1] == 0
    assert res["rebuilds"] >= 1 and res["epoch"] >= 1 and res["members"] == [0, 1]
    assert res["done"] == [True, True]
    assert res["requeued"] >= 1
    # at-least-once: every image of both jobs was served
    assert res["c1"]["ResNet50"]["query_count"] >= 96 and res["c1"]["InceptionV3"]["query_count"] >= 96


def test_coordinator_two_steps_in_flight_requeue_order():
    """Pipelined service: steps k-1 and k are both in flight; a failure requeues
    both at the queue front in their original order; completion is per step."""
    from distributed_machine_learning_amd.parallel.dataplane import F_BATCH
    from distributed_machine_learning_amd.parallel.service import CollectiveCoordinator

    c = CollectiveCoordinator({"ResNet50": 4, "InceptionV3": 4}, {"ResNet50": 64, "InceptionV3": 64})
    c.submit("ResNet50", 16)                       # 4 batches of 4
    t0 = c.next_table([0])
    t1 = c.next_table([0])
    assert sorted(c.inflight) == [0, 1] and c.steps == 2
    first = [int(t0[0, F_BATCH]), int(t1[0, F_BATCH])]
    assert c.requeue_inflight() == 2 and not c.inflight
    t2 = c.next_table([0])
    t3 = c.next_table([0])
    assert [int(t2[0, F_BATCH]), int(t3[0, F_BATCH])] == first
    c.complete([0], None, step=2)                  # out-of-order completion is per step
    assert sorted(c.inflight) == [3]
    c.complete([0], None)
    assert not c.inflight and c.metrics.c1()["ResNet50"]["query_count"] == 8
