"""Fused ResNet stem kernel (csrc/kernels/stem_fused.hip) on the GPU:
uint8 -> preprocess -> conv 7x7/2 + ReLU -> max pool 3x3/2 in one launch.

* against a plain-PyTorch fp32 reference of the same op chain (input and
  weights pre-rounded to bf16; conv output rounded to bf16 before the pool,
  the unfused engine's rounding point), over square / resized / odd shapes and
  both preprocess modes;
* inside the engine: the fused plan's pool1 output and logits equal the
  unfused three-launch plan's (fuse_stem=False)."""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from distributed_machine_learning_amd import _native as N  # noqa: E402
from distributed_machine_learning_amd import ops  # noqa: E402
from distributed_machine_learning_amd.models import build_model  # noqa: E402
from distributed_machine_learning_amd.models.engine import Engine, _r, pack_conv_weight, pair_pack_kernel  # noqa: E402
from distributed_machine_learning_amd.models.oracle import preprocess_reference  # noqa: E402


def _bf(x):
    return x.to(torch.bfloat16).float()


def _rel(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


@pytest.mark.parametrize("n,hs,ws,out_hw,mode", [
    (2, 224, 224, (224, 224), "caffe"),   # the ResNet50 shape (56x56 pool grid = 8x7 full blocks)
    (3, 300, 169, (224, 224), "caffe"),   # reference testfiles/ JPEG sizes: nearest resize in the patch fill
    (2, 64, 80, (61, 47), "tf"),          # partial blocks at the bottom/right edges
    (2, 61, 47, (61, 47), "tf"),          # identity resize (16-B pair loads) with partial edge blocks
    (1, 20, 20, (9, 9), "caffe"),         # image smaller than one block
])
def test_fused_stem_matches_fp32(n, hs, ws, out_hw, mode):
    torch.manual_seed(0)
    imgs = torch.randint(0, 256, (n, hs, ws, 3), dtype=torch.uint8)
    k = _bf(torch.randn(7, 7, 3, 64) * (2.0 / 147) ** 0.5)  # HWIO
    b = torch.randn(64) * 0.1
    x = _bf(preprocess_reference(imgs, out_hw, mode))
    ref = F.conv2d(x, k.permute(3, 2, 0, 1), b, stride=2, padding=3)
    ref = F.max_pool2d(_bf(F.relu(ref)), 3, 2, 1).permute(0, 2, 3, 1)
    wp = torch.from_numpy(pack_conv_weight(pair_pack_kernel(k.numpy()), 8, 256, 256)).to(torch.bfloat16).cuda()
    y = ops.resnet_stem(imgs.cuda(), wp, b.cuda(), out_hw, mode)
    torch.cuda.synchronize()
    got = y.float().cpu()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    rel = _rel(got, ref)
    assert rel < 1e-2, rel


@pytest.mark.parametrize("n,hs,ws,out_hw", [(2, 224, 224, (224, 224)), (2, 64, 80, (61, 47)), (1, 20, 20, (9, 9))])
def test_fused_stem_folded_1x1_matches_fp32(n, hs, ws, out_hw):
    """Step 5 of the stem kernel: the next 1x1 conv (ResNet50 conv2_block1_1, 64 -> 64 + ReLU)
    on the pooled tile in LDS; the pooled tensor is still written."""
    torch.manual_seed(1)
    imgs = torch.randint(0, 256, (n, hs, ws, 3), dtype=torch.uint8)
    k = _bf(torch.randn(7, 7, 3, 64) * (2.0 / 147) ** 0.5)
    b = torch.randn(64) * 0.1
    k4 = _bf(torch.randn(64, 64) * (2.0 / 64) ** 0.5)  # [cout][cin]
    b4 = torch.randn(64) * 0.1
    x = _bf(preprocess_reference(imgs, out_hw, "caffe"))
    pool = F.max_pool2d(_bf(F.relu(F.conv2d(x, k.permute(3, 2, 0, 1), b, stride=2, padding=3))), 3, 2, 1)
    pool = _bf(pool).permute(0, 2, 3, 1)
    zref = F.relu(pool @ k4.T + b4)
    wp = torch.from_numpy(pack_conv_weight(pair_pack_kernel(k.numpy()), 8, 256, 256)).to(torch.bfloat16).cuda()
    y, z = ops.resnet_stem(imgs.cuda(), wp, b.cuda(), out_hw, "caffe", w4=k4.to(torch.bfloat16).cuda(), b4=b4.cuda())
    torch.cuda.synchronize()
    assert _rel(y.float().cpu(), pool) < 1e-2
    assert _rel(z.float().cpu(), zref) < 1e-2, _rel(z.float().cpu(), zref)


def test_fused_stem_bad_shape_raises():
    wp = torch.zeros(64, 128, dtype=torch.bfloat16, device="cuda")  # ldw < 224
    with pytest.raises(Exception):
        ops.resnet_stem(torch.zeros(1, 32, 32, 3, dtype=torch.uint8, device="cuda"), wp,
                        torch.zeros(64, device="cuda"), (32, 32))


@pytest.mark.parametrize("fold", ["1", "0"])
def test_engine_fused_stem_equals_unfused(fold, monkeypatch):
    monkeypatch.setenv("DML_FOLD_STEM_1X1", fold)
    g, w = build_model("ResNet50", seed=7, calibrate=True)
    imgs = torch.randint(0, 256, (2, 224, 224, 3), dtype=torch.uint8, device="cuda")
    ef = Engine(g, w, batch=2, reuse_buffers=False)
    eu = Engine(g, w, batch=2, fuse_stem=False, reuse_buffers=False)
    assert ef.stem_pool is not None and eu.stem_pool is None and eu.stem_1x1 is None
    assert (ef.stem_1x1 is not None) == (fold == "1")
    want = "preprocess+conv1_conv+pool1_pool" + ("+conv2_block1_1_conv" if fold == "1" else "")
    assert ef.op_names[0] == want and len(ef.op_names) == len(eu.op_names) - 2 - (fold == "1")
    if fold == "1":  # the folded conv's output never shares a buffer with the pooled tensor it reads
        er = Engine(g, w, batch=2)
        assert er.buf[er.stem_1x1.out].data_ptr() != er.buf[er.stem_pool.out].data_ptr()
    ef.infer(imgs)
    eu.infer(imgs)
    torch.cuda.synchronize()
    # the pool output may live in a channel slice of a concat buffer (shortcut merge)
    p = next(n for n in ef.g.nodes if getattr(n, "name", "") == "pool1_pool")
    pf = ef.view(p.out)[..., p.out_coff:p.out_coff + 64].float()
    pu = eu.view(p.out)[..., p.out_coff:p.out_coff + 64].float()
    assert (pf - pu).abs().max().item() <= 1e-2 * pu.abs().max().item()
    zf, zu = ef.view("conv2_block1_1").float(), eu.view("conv2_block1_1").float()
    assert (zf - zu).abs().max().item() <= 1e-2 * zu.abs().max().item()
    assert _rel(ef.buf[g.logits].cpu(), eu.buf[g.logits].cpu()) < 2e-2


@pytest.mark.parametrize("n,hs,ws,out_hw,mode", [
    (2, 299, 299, (299, 299), "tf"),      # the InceptionV3 shape (147x147 conv2 grid, partial edge tiles)
    (2, 300, 169, (299, 299), "tf"),      # nearest resize from a reference testfiles/ JPEG size
    (1, 50, 60, (41, 39), "caffe"),       # small odd image, several partial tiles
    (3, 41, 39, (41, 39), "caffe"),       # identity resize (16-B pair loads), odd width
])
def test_fused_inception_stem_matches_fp32(n, hs, ws, out_hw, mode):
    torch.manual_seed(1)
    imgs = torch.randint(0, 256, (n, hs, ws, 3), dtype=torch.uint8)
    k1 = _bf(torch.randn(3, 3, 3, 32) * (2.0 / 27) ** 0.5)
    b1 = torch.randn(32) * 0.1
    k2 = _bf(torch.randn(3, 3, 32, 32) * (2.0 / 288) ** 0.5)
    b2 = torch.randn(32) * 0.1
    x = _bf(preprocess_reference(imgs, out_hw, mode))
    t = _bf(F.relu(F.conv2d(x, k1.permute(3, 2, 0, 1), b1, stride=2)))  # conv1 output rounded to bf16 (LDS tile)
    ref = F.relu(F.conv2d(t, k2.permute(3, 2, 0, 1), b2)).permute(0, 2, 3, 1)
    w1 = torch.from_numpy(pack_conv_weight(pair_pack_kernel(k1.numpy()), 8, 256, 64)).to(torch.bfloat16).cuda()
    w2 = torch.from_numpy(pack_conv_weight(k2.numpy(), 32, 256, 320)).to(torch.bfloat16).cuda()
    y = ops.inception_stem(imgs.cuda(), w1, b1.cuda(), w2, b2.cuda(), out_hw, mode)
    torch.cuda.synchronize()
    got = y.float().cpu()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    rel = _rel(got, ref)
    assert rel < 1e-2, rel


def test_engine_fused_inception_stem_equals_unfused():
    g, w = build_model("InceptionV3", seed=7, calibrate=True)
    imgs = torch.randint(0, 256, (2, 299, 299, 3), dtype=torch.uint8, device="cuda")
    ef = Engine(g, w, batch=2, reuse_buffers=False)
    eu = Engine(g, w, batch=2, fuse_stem=False, reuse_buffers=False)
    assert ef.stem_conv2 is not None and eu.stem_conv2 is None
    # the stem conv + conv2d_2 fold into op 0; conv2d_3 + max_pooling2d_1 (+ the 1x1 conv2d_4
    # applied to the pooled tile in LDS, DML_FOLD_POOL_1X1) into one conv+pool op
    folded = bool(ef.conv_pool_1x1)
    assert ef.op_names[0].startswith("preprocess+") and len(ef.op_names) == len(eu.op_names) - 3 - folded
    assert list(ef.conv_pools.values())[0].out == "stem_pool1"
    ef.infer(imgs)
    eu.infer(imgs)
    torch.cuda.synchronize()
    # with the fold the pooled tile never leaves LDS: compare the folded 1x1's output instead
    last = list(ef.conv_pool_1x1.values())[0].out if folded else "stem_pool1"
    for name in (ef.stem_conv2.out, last):
        pf, pu = ef.view(name).float(), eu.view(name).float()
        assert (pf - pu).abs().max().item() <= 1e-2 * pu.abs().max().item(), name
    assert _rel(ef.buf[g.logits].cpu(), eu.buf[g.logits].cpu()) < 5e-2


@pytest.mark.parametrize("n,h,w,cbuf", [(2, 147, 147, 32), (1, 20, 23, 32), (1, 9, 9, 40)])
def test_conv3x3_pool_matches_fp32(n, h, w, cbuf):
    torch.manual_seed(2)
    x = _bf(torch.randn(n, cbuf, h, w).clamp(min=0))
    k = _bf(torch.randn(3, 3, 32, 64) * (2.0 / 288) ** 0.5)
    b = torch.randn(64) * 0.1
    conv = _bf(F.relu(F.conv2d(x[:, :32], k.permute(3, 2, 0, 1), b, padding=1)))
    ref = F.max_pool2d(conv, 3, 2).permute(0, 2, 3, 1)
    wp = torch.from_numpy(pack_conv_weight(k.numpy(), 32, 256, 320)).to(torch.bfloat16).cuda()
    y = ops.conv3x3_pool(x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).cuda(), wp, b.cuda())
    torch.cuda.synchronize()
    got = y.float().cpu()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert _rel(got, ref) < 1e-2


@pytest.mark.parametrize("n,h,w,c4", [(1, 147, 147, 80), (2, 20, 23, 80), (1, 9, 9, 32), (1, 35, 19, 128)])
def test_conv3x3_pool_folded_1x1(n, h, w, c4):
    """conv2d_3 + max_pooling2d_1 + conv2d_4 (1x1 64 -> c4 + ReLU) as ONE kernel: the pooled
    tile never leaves LDS; edge blocks (partial pool tiles) included."""
    torch.manual_seed(9)
    x = _bf(torch.randn(n, 32, h, w).clamp(min=0))
    k = _bf(torch.randn(3, 3, 32, 64) * (2.0 / 288) ** 0.5)
    b = torch.randn(64) * 0.1
    w4 = _bf(torch.randn(c4, 64) * (2.0 / 64) ** 0.5)
    b4 = torch.randn(c4) * 0.1
    pool = _bf(F.max_pool2d(_bf(F.relu(F.conv2d(x, k.permute(3, 2, 0, 1), b, padding=1))), 3, 2))
    ref = F.relu(F.conv2d(pool, w4.view(c4, 64, 1, 1), b4)).permute(0, 2, 3, 1)
    wp = torch.from_numpy(pack_conv_weight(k.numpy(), 32, 256, 320)).to(torch.bfloat16).cuda()
    w4p = torch.zeros(max(c4, 64), 64)
    w4p[:c4] = w4
    y = ops.conv3x3_pool(x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).cuda(), wp, b.cuda(),
                         w4p.to(torch.bfloat16).cuda(), b4.cuda(), c4)
    torch.cuda.synchronize()
    got = y.float().cpu()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert _rel(got, ref) < 1e-2


def test_engine_folds_pool_1x1_into_conv_pool():
    """InceptionV3: conv2d_3 + max_pooling2d_1 + conv2d_4 run as one plan op and the
    forward matches the engine without the fold."""
    import os

    g, w = build_model("InceptionV3", seed=3, calibrate=True)
    imgs = torch.randint(0, 256, (2, 299, 299, 3), dtype=torch.uint8, device="cuda")
    ef = Engine(g, w, batch=2)
    os.environ["DML_FOLD_POOL_1X1"] = "0"
    try:
        eu = Engine(g, w, batch=2)
    finally:
        del os.environ["DML_FOLD_POOL_1X1"]
    assert ef.conv_pool_1x1 and not eu.conv_pool_1x1
    assert any(name.endswith("+conv2d_4") for name in ef.op_names)
    ef.infer(imgs)
    eu.infer(imgs)
    torch.cuda.synchronize()
    assert torch.equal(ef.result.cpu(), eu.result.cpu()) or _rel(ef.buf[g.logits].cpu(), eu.buf[g.logits].cpu()) < 2e-2


@pytest.mark.parametrize("c,m", [(256, 64 * 7), (256, 1000), (256, 3 * 56 * 56), (512, 1000), (512, 2 * 28 * 28),
                                 (1024, 999), (1024, 2 * 14 * 14)])
def test_expand_reduce_matches_fp32(c, m):
    torch.manual_seed(3)
    f = c // 4
    x = _bf(torch.randn(m, f).clamp(min=0))
    res = _bf(torch.randn(m, c))
    w3 = _bf(torch.randn(c, f) * (2.0 / f) ** 0.5)
    b3 = torch.randn(c) * 0.1
    w1 = _bf(torch.randn(f, c) * (2.0 / c) ** 0.5)
    b1 = torch.randn(f) * 0.1
    y_ref = _bf(F.relu(x @ w3.T + b3 + res))  # the engine's rounding point
    z_ref = F.relu(y_ref @ w1.T + b1)
    w1p = torch.zeros(max(f, 64), c)  # packed weights: rows padded like pack_weight
    w1p[:f] = w1
    y, z = ops.expand_reduce(x.to(torch.bfloat16).cuda(), w3.to(torch.bfloat16).cuda(), b3.cuda(),
                             res.to(torch.bfloat16).cuda(), w1p.to(torch.bfloat16).cuda(), b1.cuda())
    torch.cuda.synchronize()
    assert _rel(y.float().cpu(), y_ref) < 1e-2
    assert _rel(z.float().cpu(), z_ref) < 1e-2


@pytest.mark.parametrize("maxc,chain,merged,pairs", [(256, "0", "0", 2), (256, "1", "0", 4), (256, "2", "0", 8),
                                                     (1024, "0", "0", 8), (256, "1", "1", 5), (256, "1", "", 5)])
def test_engine_fused_blocks_equal_unfused(maxc, chain, merged, pairs, monkeypatch):
    """DML_CHAIN=1 (default) adds stage 3's boundaries (C = 512, chained kernel), 2 also stage 4's;
    DML_CHAIN_MERGED=1 routes stage 2's merged entry (K = 2F) to the chained kernel; stage 3's merged
    entry (conv3_block1_3 + _0) reads [x ; s] with K = F + 256 = 3F, which the chained kernel's
    merged form (K = 2F) does not take, so it stays two launches. Stage 2's last expand
    (conv2_block3_3, its shortcut stored compactly by the boundary before) is chained with stage
    3's first reduce (256 -> 128) in every case (DML_CHAIN_STAGE_END, default on)."""
    monkeypatch.setenv("DML_FUSED_BLOCKS_MAXC", str(maxc))
    monkeypatch.setenv("DML_CHAIN", chain)
    if merged:
        monkeypatch.setenv("DML_CHAIN_MERGED", merged)
    else:  # the default: the merged stage-2 entry on the chained kernel
        monkeypatch.delenv("DML_CHAIN_MERGED", raising=False)
    g, w = build_model("ResNet50", seed=8, calibrate=True)
    imgs = torch.randint(0, 256, (2, 224, 224, 3), dtype=torch.uint8, device="cuda")
    # no buffer recycling: intermediate tensors are compared after the whole forward
    ef = Engine(g, w, batch=2, reuse_buffers=False)
    eu = Engine(g, w, batch=2, fuse_blocks=False, reuse_buffers=False)
    # block boundaries: stage 2's first (its expand absorbed the projection shortcut,
    # models/optimize.py: K = 2F, no residual) and second; stage 3: 2, stage 4: 4 (the merged
    # first expands of stages 3-5 and stage 5, C = 2048, are not fused)
    # (DML_CHAIN_MERGED=0: the merged stage-2 entry runs as its two launches — the r1 kernel
    # that used to take it was removed in r5)
    want = (["conv2_block1_3_conv+conv2_block1_0_conv"] if merged != "0" else []) + [
        f"conv{s}_block{k}_3_conv" for s, nb in ((2, 3), (3, 4), (4, 6)) for k in range(2, nb)]
    want = want[:pairs - 1] + ["conv2_block3_3_conv"]
    assert sorted(ef.exp_red) == sorted(want) and not eu.exp_red
    assert ef.exp_red["conv2_block3_3_conv"].name == "conv3_block1_1_conv"
    # the last fused boundary of each stage feeds only the stride-2 shortcut besides its reduce
    assert "conv2_block2_out" in ef.ysub and not eu.ysub
    assert len(ef.op_names) == len(eu.op_names) - pairs
    # the fused kernel writes the reduce output while reading the expand inputs: never
    # aliased, also under liveness-based buffer recycling
    er = Engine(g, w, batch=2)
    for e_name, r in er.exp_red.items():
        e = next(n for n in er.g.nodes if n.name == e_name)
        srcs = [er.buf[e.inp].data_ptr()] + ([er.buf[e.residual].data_ptr()] if e.residual else [])
        assert er.buf[r.out].data_ptr() not in srcs
    ef.infer(imgs)
    eu.infer(imgs)
    torch.cuda.synchronize()
    # (stage-final block outputs now live in the next stage's concat buffer, not under their own name)
    for name in ("conv2_block1_out", "conv2_block2_1", "conv2_block2_out", "conv2_block3_1", "conv3_block1_1",
                 "conv3_block1_2", "conv3_block2_1", "conv3_block3_out", "conv4_block2_1", "conv4_block6_1",
                 "conv4_block5_out"):
        pf, pu = ef.view(name).float(), eu.view(name).float()
        if name in ef.ysub:  # stored compactly: only the pixels the stride-2 shortcut reads
            b, h, w, cb = pf.shape
            pf = ef.buf[name].view(-1)[: b * (h // 2) * (w // 2) * cb].view(b, h // 2, w // 2, cb).float()
            pu = pu[:, ::2, ::2]
        assert (pf - pu).abs().max().item() <= 2e-2 * pu.abs().max().item(), name
    assert _rel(ef.buf[g.logits].cpu(), eu.buf[g.logits].cpu()) < 5e-2


@pytest.mark.parametrize("c,m", [(256, 64 * 7), (256, 1000), (256, 3 * 56 * 56), (512, 300), (512, 2 * 28 * 28)])
def test_expand_reduce_merged_shortcut_matches_fp32(c, m):
    """K = 2F, no residual: a stage's entry after the projection-shortcut merge (chained
    kernel: C = 256 and 512)."""
    torch.manual_seed(4)
    f = c // 4
    x = _bf(torch.randn(m, 2 * f))
    w3 = _bf(torch.randn(c, 2 * f) * (2.0 / (2 * f)) ** 0.5)
    b3 = torch.randn(c) * 0.1
    w1 = _bf(torch.randn(f, c) * (2.0 / c) ** 0.5)
    b1 = torch.randn(f) * 0.1
    y_ref = _bf(F.relu(x @ w3.T + b3))
    z_ref = F.relu(y_ref @ w1.T + b1)
    w1p = torch.zeros(max(f, 64), c)
    w1p[:f] = w1
    y, z = ops.expand_reduce(x.to(torch.bfloat16).cuda(), w3.to(torch.bfloat16).cuda(), b3.cuda(), None,
                             w1p.to(torch.bfloat16).cuda(), b1.cuda(), c=c)
    torch.cuda.synchronize()
    assert _rel(y.float().cpu(), y_ref) < 1e-2
    assert _rel(z.float().cpu(), z_ref) < 1e-2


def test_expand_reduce_subsampled_y():
    """ysub = 2: Y stored only at even (h, w), compactly; Z complete."""
    torch.manual_seed(5)
    n, h, w, c, f = 2, 10, 12, 256, 64
    m = n * h * w
    x = _bf(torch.randn(m, f).clamp(min=0))
    res = _bf(torch.randn(m, c))
    w3 = _bf(torch.randn(c, f) * (2.0 / f) ** 0.5)
    b3 = torch.randn(c) * 0.1
    w1 = _bf(torch.randn(f, c) * (2.0 / c) ** 0.5)
    b1 = torch.randn(f) * 0.1
    y_ref = _bf(F.relu(x @ w3.T + b3 + res))
    z_ref = F.relu(y_ref @ w1.T + b1)
    w1p = torch.zeros(64, c)
    w1p[:f] = w1
    xd, rd = x.to(torch.bfloat16).cuda(), res.to(torch.bfloat16).cuda()
    y = torch.full((m, c), -7.0, device="cuda", dtype=torch.bfloat16)
    z = torch.empty((m, f), device="cuda", dtype=torch.bfloat16)
    w3d, w1d = w3.to(torch.bfloat16).cuda(), w1p.to(torch.bfloat16).cuda()
    b3d, b1d = b3.cuda(), b1.cuda()
    a = N.ExpandReduceArgs(xd.data_ptr(), w3d.data_ptr(), b3d.data_ptr(), rd.data_ptr(), y.data_ptr(), w1d.data_ptr(),
                           b1d.data_ptr(), z.data_ptr(), m, f, f, c, c, c, f, c, f, 2, h, w)
    N.check(N.lib().dml_expand_reduce(C.byref(a), N.stream_ptr()), "expand_reduce ysub")
    torch.cuda.synchronize()
    q = n * (h // 2) * (w // 2)
    want = y_ref.view(n, h, w, c)[:, ::2, ::2].reshape(q, c)
    assert _rel(y[:q].float().cpu(), want) < 1e-2
    assert (y[q:].float() == -7.0).all()  # nothing stored past the compact tensor
    assert _rel(z.float().cpu(), z_ref) < 1e-2


@pytest.mark.parametrize("c,m", [(512, 256), (512, 300), (512, 2 * 28 * 28), (512, 7 * 28 * 28 + 13),
                                 (1024, 64), (1024, 77), (1024, 3 * 14 * 14 + 5)])
def test_expand_reduce_chain(c, m):
    """C = 512 / 1024 go to the chained-GEMM kernel (expand_reduce_chain.hip): Y written
    once, Z from Y in registers; workgroup tails and several workgroups."""
    torch.manual_seed(6)
    f = c // 4
    x = _bf(torch.randn(m, f).clamp(min=0))
    res = _bf(torch.randn(m, c))
    w3 = _bf(torch.randn(c, f) * (2.0 / f) ** 0.5)
    b3 = torch.randn(c) * 0.1
    w1 = _bf(torch.randn(f, c) * (2.0 / c) ** 0.5)
    b1 = torch.randn(f) * 0.1
    y_ref = _bf(F.relu(x @ w3.T + b3 + res))
    z_ref = F.relu(y_ref @ w1.T + b1)
    y, z = ops.expand_reduce(x.to(torch.bfloat16).cuda(), w3.to(torch.bfloat16).cuda(), b3.cuda(),
                             res.to(torch.bfloat16).cuda(), w1.to(torch.bfloat16).cuda(), b1.cuda())
    torch.cuda.synchronize()
    assert _rel(y.float().cpu(), y_ref) < 1e-2
    assert _rel(z.float().cpu(), z_ref) < 1e-2


@pytest.mark.parametrize("c", [512, 1024])
def test_expand_reduce_chain_subsampled_y(c):
    torch.manual_seed(7)
    n, h, w = 3, 14, 10
    f = c // 4
    m = n * h * w
    x = _bf(torch.randn(m, f).clamp(min=0))
    res = _bf(torch.randn(m, c))
    w3 = _bf(torch.randn(c, f) * (2.0 / f) ** 0.5)
    b3 = torch.randn(c) * 0.1
    w1 = _bf(torch.randn(f, c) * (2.0 / c) ** 0.5)
    b1 = torch.randn(f) * 0.1
    y_ref = _bf(F.relu(x @ w3.T + b3 + res))
    z_ref = F.relu(y_ref @ w1.T + b1)
    xd, rd = x.to(torch.bfloat16).cuda(), res.to(torch.bfloat16).cuda()
    y = torch.full((m, c), -7.0, device="cuda", dtype=torch.bfloat16)
    z = torch.empty((m, f), device="cuda", dtype=torch.bfloat16)
    w3d, w1d = w3.to(torch.bfloat16).cuda(), w1.to(torch.bfloat16).cuda()
    b3d, b1d = b3.cuda(), b1.cuda()
    a = N.ExpandReduceArgs(xd.data_ptr(), w3d.data_ptr(), b3d.data_ptr(), rd.data_ptr(), y.data_ptr(), w1d.data_ptr(),
                           b1d.data_ptr(), z.data_ptr(), m, f, f, c, c, c, f, c, f, 2, h, w)
    assert N.lib().dml_chain_supported(C.byref(a)) == 1
    N.check(N.lib().dml_expand_reduce(C.byref(a), N.stream_ptr()), "expand_reduce chain ysub")
    torch.cuda.synchronize()
    q = n * (h // 2) * (w // 2)
    want = y_ref.view(n, h, w, c)[:, ::2, ::2].reshape(q, c)
    assert _rel(y[:q].float().cpu(), want) < 1e-2
    assert (y[q:].float() == -7.0).all()
    assert _rel(z.float().cpu(), z_ref) < 1e-2


@pytest.mark.parametrize("m,f", [(128, 64), (300, 64), (2 * 28 * 28, 64), (5 * 28 * 28 + 7, 64),
                                 (64, 128), (3 * 14 * 14 + 5, 128)])
def test_expand_reduce_chain_stage_end(m, f):
    """A stage's last boundary (chained kernel, fz = 2F): y = relu(x W3 + b3 + res) (F -> 4F)
    stored into channels [2F, 6F) of a 6F-wide concat buffer, z = relu(y W1 + b1) (4F -> 2F)."""
    torch.manual_seed(9)
    c, fz, ldy, coff = 4 * f, 2 * f, 6 * f, 2 * f
    x = _bf(torch.randn(m, f).clamp(min=0))
    res = _bf(torch.randn(m, c))
    w3 = _bf(torch.randn(c, f) * (2.0 / f) ** 0.5)
    b3 = torch.randn(c) * 0.1
    w1 = _bf(torch.randn(fz, c) * (2.0 / c) ** 0.5)
    b1 = torch.randn(fz) * 0.1
    y_ref = _bf(F.relu(x @ w3.T + b3 + res))
    z_ref = F.relu(y_ref @ w1.T + b1)
    xd, rd = x.to(torch.bfloat16).cuda(), res.to(torch.bfloat16).cuda()
    y = torch.full((m, ldy), -7.0, device="cuda", dtype=torch.bfloat16)
    z = torch.empty((m, fz), device="cuda", dtype=torch.bfloat16)
    w3d, w1d = w3.to(torch.bfloat16).cuda(), w1.to(torch.bfloat16).cuda()
    b3d, b1d = b3.cuda(), b1.cuda()
    a = N.ExpandReduceArgs(xd.data_ptr(), w3d.data_ptr(), b3d.data_ptr(), rd.data_ptr(), y.data_ptr() + 2 * coff,
                           w1d.data_ptr(), b1d.data_ptr(), z.data_ptr(), m, f, f, c, ldy, c, fz, c, f)
    a.fz = fz
    assert N.lib().dml_chain_supported(C.byref(a)) == 1
    N.check(N.lib().dml_expand_reduce(C.byref(a), N.stream_ptr()), "expand_reduce stage end")
    torch.cuda.synchronize()
    assert _rel(y[:, coff:].float().cpu(), y_ref) < 1e-2
    assert (y[:, :coff].float() == -7.0).all()  # the other slice of the concat is untouched
    assert _rel(z.float().cpu(), z_ref) < 1e-2
    y2, z2 = ops.expand_reduce(xd, w3d, b3d, rd, w1d, b1d, fz=fz)  # the torch-facing wrapper
    torch.cuda.synchronize()
    assert _rel(y2.float().cpu(), y_ref) < 1e-2 and _rel(z2.float().cpu(), z_ref) < 1e-2
