"""GPU tests of the serving paths the benches time (RCCL at world 1):

* ServingPipeline (bench.py's timed loop: dispatch broadcast, double-buffered
  H2D slots, SplitEngine hipGraph forward, RCCL gather) over 6 steps with
  distinct images per step == Engine.infer of each batch, bit-exact;
* the collective service (replicated coordinator + GpuRankBackend + output
  writer) over RCCL: every output file present and equal to the engine; a C3
  batch larger than the engine's batch runs as several passes (not truncated);
* the host-mode GpuBackend.predict (bucketed engines, pinned staging);
* PinnedImageStore.h2d_indices (coalesced runs);
* RCCL failure semantics: explicit communicator abort, re-init of a new epoch
  over the FileStore rendezvous, then a collective that succeeds.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def rccl_world1(monkeypatch):
    import torch.distributed as dist

    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_free_port()))
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("LOCAL_RANK", "0")
    yield
    if dist.is_initialized():
        dist.destroy_process_group()


def _split_ref(g, w, imgs, half, parts=2):
    """Engine(batch=half) on each of the ``parts`` slices of imgs -> packed
    [2, parts*half, 5] (the SplitEngine reference used by test_engine_gpu)."""
    from distributed_machine_learning_amd.models.engine import Engine

    e = Engine(g, w, batch=half)
    out = []
    for h in range(parts):
        e.infer(imgs[h * half:(h + 1) * half].cuda())
        torch.cuda.synchronize()
        out.append(e.result.clone().cpu())
    return torch.cat(out, dim=1)


@pytest.mark.parametrize("splits,streams,lookahead,lag", [(2, 0, 2, None), (8, 2, 2, None), (2, 0, 1, None),
                                                          (2, 0, 2, 1), (8, 2, 2, 1)])
def test_serving_pipeline_matches_engine(rccl_world1, splits, streams, lookahead, lag):
    """splits 8 on 2 streams: eight graph captures; captured lazily inside the
    loop they once met the RCCL watchdog querying an event on a capturing stream
    (hipErrorCapturedEvent), hence Engine.capture() before the first collective.
    lag 1: the world > 1 schedule (result gather of batch k on the comm stream after
    forward k+1, rows through the send ring) forced at world 1 on the real engines."""
    from distributed_machine_learning_amd.models import build_model
    from distributed_machine_learning_amd.models.engine import SplitEngine
    from distributed_machine_learning_amd.parallel.dataplane import DESC_FIELDS, DataPlane, init_process_group
    from distributed_machine_learning_amd.parallel.pipeline import ServingPipeline
    from distributed_machine_learning_amd.parallel.staging import PinnedImageStore

    rank, world, local = init_process_group()
    dev = torch.device("cuda", local)
    B, steps = 16, 6
    g, w = build_model("ResNet50", seed=0)
    eng = SplitEngine(g, w, batch=B, device=str(dev), src_slots=2, splits=splits, streams=streams)
    store = PinnedImageStore(capacity=steps * B, hw=g.input_hw)
    store.fill_synthetic(seed=3)
    dp = DataPlane(dev, result_shape=(2, B, 5))
    got = {}
    pipe = ServingPipeline(eng, store, dp, use_graph=True, on_results=lambda rec: got.__setitem__(rec.step, rec.results[0]),
                           lookahead=lookahead, gather_lag=lag)
    assert pipe.gather_lag == (lag or 0)

    def table(k):
        t = np.zeros((world, DESC_FIELDS), np.int64)
        t[0] = (31, k, 0, k * B, B, 0)
        return t

    pipe.run(steps, table)
    assert sorted(got) == list(range(steps))
    for k in range(steps):
        ref = _split_ref(g, w, torch.from_numpy(store.array[k * B:(k + 1) * B].copy()), B // splits, splits)
        assert torch.equal(got[k], ref), f"step {k} differs"


def test_pinned_h2d_indices():
    from distributed_machine_learning_amd.parallel.staging import PinnedImageStore

    st = PinnedImageStore(capacity=12, hw=(8, 8))
    st.fill_synthetic(seed=1)
    idx = [3, 4, 5, 0, 9, 10, 2]
    dst = torch.empty((len(idx), 8, 8, 3), dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    st.h2d_indices(dst, idx, s)
    s.synchronize()
    assert torch.equal(dst.cpu(), torch.from_numpy(st.array[idx]))
    st.h2d(dst[:5], 10, 5, s)  # wrapping range
    s.synchronize()
    assert torch.equal(dst[:5].cpu(), torch.from_numpy(st.array[[10, 11, 0, 1, 2]]))


def test_gpu_backend_predict_buckets():
    from distributed_machine_learning_amd.models import build_model
    from distributed_machine_learning_amd.models.engine import Engine
    from distributed_machine_learning_amd.serving.inference import GpuBackend

    be = GpuBackend(max_batch=64, quantum=32)
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (70, 224, 224, 3), dtype=np.uint8)  # 64 + one 32-bucket pass of 6
    idx, p = be.predict("ResNet50", imgs)
    assert sorted(k[1] for k in be._engines) == [32, 64]
    g, w = build_model("ResNet50", seed=0)
    ref = Engine(g, w, batch=64)
    ref.infer(torch.from_numpy(imgs[:64]).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(idx[:64], ref.top_idx.cpu().numpy())
    assert np.array_equal(p[:64], ref.top_p.cpu().numpy())
    r32 = Engine(g, w, batch=32)
    src = np.zeros((32, 224, 224, 3), np.uint8)
    src[:6] = imgs[64:]
    r32.infer(torch.from_numpy(src).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(idx[64:], r32.top_idx.cpu().numpy()[:6])


def test_collective_service_rccl_world1_outputs(tmp_path):
    from distributed_machine_learning_amd.models import build_model
    from distributed_machine_learning_amd.parallel.elastic import ElasticGroup
    from distributed_machine_learning_amd.parallel.service import (CollectiveService, GpuRankBackend, OutputWriter,
                                                                   ReplicatedCoordinator)
    from distributed_machine_learning_amd.utils.labels import load_class_index

    dev = torch.device("cuda", 0)
    eg = ElasticGroup(0, 1, store_path=str(tmp_path / "rdzv"), backend="nccl", device=dev, timeout_s=120)
    try:
        bs = {"ResNet50": 16, "InceptionV3": 8}
        be = GpuRankBackend(dev, bs, cap=32, arena_images=256, n_synth=64)
        assert be.arenas["ResNet50"].arena.device.type == "cuda"  # the image store lives in HBM
        coord = ReplicatedCoordinator(bs, cap=32, host_tag="gpu")
        writer = OutputWriter(str(tmp_path / "out"), host_tag="gpu")
        svc = CollectiveService(eg, be, coord, writer=writer, on_device=True)
        svc.submit_local("ResNet50", 40)        # 16 + 16 + 8
        svc.submit_local("InceptionV3", 20)     # 8 + 8 + 4
        svc.set_batch_size("ResNet50", 32)      # applied after the first submit's batching
        svc.submit_local("ResNet50", 32)        # one 32-image batch = 2 engine passes of 16
        svc.serve(max_steps=10 ** 6, stop_when_idle=True)
        assert [coord.jobs.jobs[j].done for j in (31, 32, 33)] == [True, True, True]
        files = sorted(os.listdir(tmp_path / "out"))
        assert len(files) == 3 + 3 + 1, files
        cls = {wnid: i for i, (wnid, _) in enumerate(load_class_index())}
        for m, job, n_img, half in (("ResNet50", 31, 40, 8), ("InceptionV3", 32, 20, 4), ("ResNet50", 33, 32, 8)):
            g, w = build_model(m, seed=0)
            arena = be.arenas[m].arena.cpu().numpy()
            doc = {}
            for f in files:
                if f.startswith(f"output_{job}_"):
                    doc.update(json.load(open(tmp_path / "out" / f)))
            assert len(doc) == n_img or job == 33  # job 33 reuses names synthetic:0..31
            names = [f"{i}" for i in range(n_img)]
            imgs = torch.from_numpy(arena[[i % 64 for i in range(n_img)]].copy())
            bsz = 32 if job == 33 else bs[m]
            for b0 in range(0, n_img, bsz):
                rows = imgs[b0:b0 + bsz]
                pad = torch.zeros((bsz, *rows.shape[1:]), dtype=torch.uint8)
                pad[:len(rows)] = rows
                if job == 33:  # two engine passes of 16 (SplitEngine halves of 8)
                    ref = torch.cat([_split_ref(g, w, pad[:16], 8), _split_ref(g, w, pad[16:], 8)], dim=1)
                else:
                    ref = _split_ref(g, w, pad, half)
                for i in range(len(rows)):
                    ent = doc[f"synthetic:{names[b0 + i]}"][0]
                    assert [cls[e[0]] for e in ent] == ref[0, i].tolist()
                    assert np.allclose([e[2] for e in ent], ref[1, i].view(torch.float32).numpy(), rtol=0, atol=0)
    finally:
        eg.close()


def test_store_images_replicated_to_hbm_and_served(tmp_path):
    """Store JPEGs -> decoded once into the HBM image store through the data
    group (RCCL) at submit -> served from HBM; control collectives on host gloo
    (the service default). Output rows == Engine.infer of the same decoded
    images; an undecodable file is reported as failed."""
    import io

    from PIL import Image

    from distributed_machine_learning_amd.models import build_model
    from distributed_machine_learning_amd.parallel.elastic import ElasticGroup
    from distributed_machine_learning_amd.parallel.service import (CollectiveService, GpuRankBackend, OutputWriter,
                                                                   ReplicatedCoordinator)
    from distributed_machine_learning_amd.serving.inference import load_image
    from distributed_machine_learning_amd.serving.output import FAILED_DOWNLOAD
    from distributed_machine_learning_amd.utils.labels import load_class_index

    rng = np.random.default_rng(0)
    blobs = {}
    for i in range(12):
        buf = io.BytesIO()
        Image.fromarray(rng.integers(0, 255, (300, 200 + 8 * i, 3), dtype=np.uint8)).save(buf, format="JPEG")
        blobs[f"{i}.jpeg"] = buf.getvalue()
    blobs["broken.jpeg"] = b"not a jpeg"
    dev = torch.device("cuda", 0)
    eg = ElasticGroup(0, 1, store_path=str(tmp_path / "rdzv"), backend="gloo", data_backend="nccl", timeout_s=120)
    try:
        bs = {"ResNet50": 8, "InceptionV3": 8}
        be = GpuRankBackend(dev, bs, cap=8, arena_images=64, n_synth=8, loader=lambda ns: {n: blobs.get(n) for n in ns})
        coord = ReplicatedCoordinator(bs, cap=8, host_tag="gpu")
        writer = OutputWriter(str(tmp_path / "out"), host_tag="gpu")
        svc = CollectiveService(eg, be, coord, writer=writer, on_device=False)
        names = sorted(blobs)
        svc.submit_local("ResNet50", images=names)
        svc.serve(max_steps=10 ** 6, stop_when_idle=True)
        st = be.arenas["ResNet50"]
        assert st.replicated == 12 and st.windows_staged >= 1   # decoded once, staged in windows
        doc = {}
        for f in os.listdir(tmp_path / "out"):
            doc.update(json.load(open(tmp_path / "out" / f)))
        assert doc["broken.jpeg"] == FAILED_DOWNLOAD
        g, w = build_model("ResNet50", seed=0)
        good = [n for n in names if n != "broken.jpeg"]
        imgs = torch.from_numpy(np.stack([load_image(blobs[n], (224, 224)) for n in good]))
        cls = {wnid: i for i, (wnid, _) in enumerate(load_class_index())}
        for b0 in range(0, len(names), 8):  # batches of 8 in submit order, failed rows computed on slot 0
            batch = names[b0:b0 + 8]
            pad = torch.zeros((8, 224, 224, 3), dtype=torch.uint8)
            for i, n in enumerate(batch):
                pad[i] = imgs[good.index(n)] if n in good else torch.from_numpy(st.arena[0].cpu().numpy())
            ref = _split_ref(g, w, pad, 4)
            for i, n in enumerate(batch):
                if n in good:
                    assert [cls[e[0]] for e in doc[n][0]] == ref[0, i].tolist(), n
    finally:
        eg.close()


def test_rccl_abort_and_new_epoch(tmp_path):
    """Explicit abort of the RCCL communicator (the path a dead peer triggers),
    re-init of epoch 1 through the FileStore rendezvous, then collectives that
    succeed on the new communicator."""
    from distributed_machine_learning_amd.parallel.elastic import ElasticGroup

    dev = torch.device("cuda", 0)
    eg = ElasticGroup(0, 1, store_path=str(tmp_path / "rdzv"), backend="nccl", device=dev, timeout_s=60)
    try:
        t = torch.arange(4, device=dev, dtype=torch.float32)
        eg.broadcast(t, 0)
        members = eg.rebuild(set())          # abort epoch 0, join epoch 1
        assert members == [0] and eg.epoch == 1 and eg.aborts == 1
        t2 = torch.ones(8, device=dev)
        eg.broadcast(t2, 0)
        bufs = [torch.empty_like(t2)]
        eg.all_gather(bufs, t2)
        torch.cuda.synchronize()
        assert torch.equal(bufs[0], t2)
        eg.barrier()
    finally:
        eg.close()


def test_job_three_times_the_arena_gpu(tmp_path):
    """One job with 3x the HBM arena's image capacity in distinct store JPEGs
    (RCCL data group, world 1): windows are staged ahead of dispatch and the oldest
    unpinned images evicted as batches complete; every image is decoded once and every
    output row equals Engine.infer of the right decoded image (a job larger
    than the arena used to kill the service)."""
    import io

    from PIL import Image

    from distributed_machine_learning_amd.models import build_model
    from distributed_machine_learning_amd.parallel.elastic import ElasticGroup
    from distributed_machine_learning_amd.parallel.service import (CollectiveService, GpuRankBackend, OutputWriter,
                                                                   ReplicatedCoordinator)
    from distributed_machine_learning_amd.serving.inference import load_image
    from distributed_machine_learning_amd.utils.labels import load_class_index

    rng = np.random.default_rng(1)
    blobs = {}
    for i in range(48):
        buf = io.BytesIO()
        Image.fromarray(rng.integers(0, 255, (256, 240 + 2 * i, 3), dtype=np.uint8)).save(buf, format="JPEG")
        blobs[f"a{i}.jpeg"] = buf.getvalue()
    loads = []

    def loader(ns):
        loads.append(list(ns))
        return {n: blobs.get(n) for n in ns}
    dev = torch.device("cuda", 0)
    eg = ElasticGroup(0, 1, store_path=str(tmp_path / "rdzv"), backend="gloo", data_backend="nccl", timeout_s=120)
    try:
        bs = {"ResNet50": 8, "InceptionV3": 8}
        be = GpuRankBackend(dev, bs, cap=8, arena_images=16, n_synth=8, loader=loader)
        st = be.arenas["ResNet50"]
        assert st.capacity == 24                      # 16 image slots (+ 8 synthetic) for a 48-image job
        coord = ReplicatedCoordinator(bs, cap=8, host_tag="gpu")
        writer = OutputWriter(str(tmp_path / "out"), host_tag="gpu")
        svc = CollectiveService(eg, be, coord, writer=writer, on_device=False)
        na = [f"a{i}.jpeg" for i in range(48)]
        svc.submit_local("ResNet50", images=na)
        svc.serve(max_steps=10 ** 6, stop_when_idle=True)
        assert st.replicated == 48 and st.evictions >= 32   # each image decoded once; slots recycled
        assert sorted(n for ns in loads for n in ns) == sorted(na)
        doc = {}
        for f in os.listdir(tmp_path / "out"):
            doc.update(json.load(open(tmp_path / "out" / f)))
        assert sorted(doc) == sorted(na)
        g, w = build_model("ResNet50", seed=0)
        cls = {wnid: i for i, (wnid, _) in enumerate(load_class_index())}
        for names in (na,):
            imgs = torch.from_numpy(np.stack([load_image(blobs[n], (224, 224)) for n in names]))
            for b0 in range(0, 48, 8):
                rows = imgs[b0:b0 + 8]
                pad = torch.zeros((8, 224, 224, 3), dtype=torch.uint8)
                pad[:len(rows)] = rows
                ref = _split_ref(g, w, pad, 4)
                for i in range(len(rows)):
                    n = names[b0 + i]
                    assert [cls[e[0]] for e in doc[n][0]] == ref[0, i].tolist(), n
                    assert np.allclose([e[2] for e in doc[n][0]], ref[1, i].view(torch.float32).numpy(),
                                       rtol=0, atol=0), n
    finally:
        eg.close()


def test_kill_pass_world4_on_one_gpu(tmp_path):
    """BASELINE config 5 on the real engines: bench.py's kill pass
    (service_bench.run_in_children) with 4 ranks sharing this GPU — each rank a child
    process running GpuRankBackend, control over gloo + shared memory — ranks 1 and 2
    killed mid-job (exit 17). The survivors rebuild twice, both jobs finish, and every
    batch's output is in the store exactly once."""
    import threading

    from distributed_machine_learning_amd.parallel import service_bench

    world, bs = 4, {"ResNet50": 64, "InceptionV3": 32}
    n_r, n_i = 64 * 48, 32 * 48
    kills = [(1, 24), (2, 48)]
    rdzv, port = str(tmp_path / "rdzv"), 20000 + os.getpid() % 20000
    recs, errs = {}, []

    def one(r):
        try:
            recs[r] = service_bench.run_in_children(r, world, 0, rdzv, port, n_r, n_i, bs, kills, timeout_s=400)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append((r, e))
    ts = [threading.Thread(target=one, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(450)
    assert not errs, errs
    rec = recs[0]
    assert rec["jobs_done"] and rec["rebuilds"] == 2 and rec["final_members"] == [0, 3]
    nb = 48 + 48
    o = rec["outputs"]
    assert o["distinct_batches_in_store"] == nb and o["listing_duplicates"] == 0, o
    # the fair-share split on the real engines (at world 1 it is degenerate):
    # with both jobs queued every split gives each model at least one of the live ranks
    splits = rec["fair_share_splits"]
    assert splits and any(s.get("ResNet50", 0) >= 1 and s.get("InceptionV3", 0) >= 1 for s in splits), splits
    assert rec["images"]["ResNet50"] >= n_r and rec["images"]["InceptionV3"] >= n_i, rec["images"]


@pytest.mark.parametrize("model", ["ResNet50", "InceptionV3"])
def test_engine_reads_arena_through_index_table(model):
    """the serving engines read a batch's images in place from the HBM
    arena through a per-slot device index table (stem kernels' ``idx``, filled from pinned
    host memory by dml_index_fetch), and write their top-5 rows straight into pinned host
    result buffers. The rows are bit-identical to the same engine configuration fed a
    gathered batch buffer."""
    from distributed_machine_learning_amd import _native as N
    from distributed_machine_learning_amd.models import build_model
    from distributed_machine_learning_amd.models.engine import SplitEngine, merge_point

    g, w = build_model(model, seed=0)
    b = 8
    dev = torch.device("cuda")
    gen = torch.Generator().manual_seed(5)
    arena = torch.randint(0, 256, (40, *g.input_hw, 3), dtype=torch.uint8, generator=gen).to(dev)
    hidx = [torch.zeros(b, dtype=torch.int32).pin_memory() for _ in range(2)]
    idx = [torch.zeros(b, dtype=torch.int32, device=dev) for _ in range(2)]
    host = [torch.full((2, b, 5), -7, dtype=torch.int32).pin_memory() for _ in range(2)]
    s = torch.cuda.Stream()
    kw = dict(batch=b, device="cuda", src_slots=2, splits=2, merge_at=merge_point(model))
    se = SplitEngine(g, w, src_tensors=[arena] * 2, src_index=idx, result_views=host, **kw)
    ref = SplitEngine(g, w, **kw)
    se.capture(s)
    ref.capture(s)
    for slot, sel in ((1, [37, 3, 3, 20, 0, 39, 11, 5]), (0, [9, 8, 7, 6, 5, 4, 3, 2])):
        hidx[slot].numpy()[:] = sel
        with torch.cuda.stream(s):
            N.check(N.lib().dml_index_fetch(hidx[slot].data_ptr(), idx[slot].data_ptr(), b, s.cuda_stream),
                    "index fetch")
            se.run(s, use_graph=True, slot=slot)
            ref.srcs[slot].copy_(arena[torch.tensor(sel, device=dev)])
            ref.run(s, use_graph=True, slot=slot)
        s.synchronize()
        assert torch.equal(host[slot], ref.results[slot].cpu()), (model, slot)
    with pytest.raises(RuntimeError, match="index table"):
        se.infer(arena[:b])
