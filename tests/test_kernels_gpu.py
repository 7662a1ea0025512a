"""Numerics of every hand-written gfx950 kernel against a plain-PyTorch fp32
reference of the same op (inputs pre-rounded to bf16 so only the kernel's
accumulation/rounding differs). Shapes cover every conv class of SURVEY §2.7:
1x1 s1/s2, 3x3, 5x5, 7x7/2 stem (Cin padded 3->8), 1x7 / 7x1 / 1x3 / 3x1,
Cin=80 (K-tile straddles taps), channel-offset concat stores, residual+ReLU,
fp32 output (FC)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from distributed_machine_learning_amd import ops  # noqa: E402


def _bf(x):
    return x.to(torch.bfloat16).float()


def _rel(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


CONV_CASES = [
    # n, h, w, cin, cout, kh, kw, stride, pad, relu, residual
    (2, 14, 14, 64, 64, 1, 1, 1, 0, True, False),
    (2, 14, 14, 256, 128, 1, 1, 2, 0, True, False),
    (2, 28, 28, 64, 256, 1, 1, 1, 0, True, True),
    (2, 9, 11, 64, 96, 3, 3, 1, 1, True, False),
    (1, 35, 35, 48, 64, 5, 5, 1, 2, True, False),
    (2, 17, 17, 128, 192, 1, 7, 1, 0, True, False),
    (2, 17, 17, 128, 192, 7, 1, 1, 0, True, False),
    (2, 8, 8, 384, 384, 1, 3, 1, 0, True, False),
    (2, 8, 8, 384, 384, 3, 1, 1, 0, True, False),
    (1, 73, 73, 80, 192, 3, 3, 1, 0, True, False),
    (2, 35, 35, 288, 384, 3, 3, 2, 0, True, False),
    (2, 7, 7, 512, 2048, 1, 1, 1, 0, False, True),
]


def _pads(kh, kw, pad):
    return (pad if kh > 1 else 0, pad if kw > 1 else 0) if pad else (0, 0)


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("cfg", [-1, 10, 11, 12, 13, 14, 15, 16, 17, 18, 23, 24, 25, 26, 27, 28, 29,
                                 30, 31, 32, 33, 34, 36, 37, 38, 39, 48, 49, 56, 57, 58, 59, 60])
def test_conv_matches_fp32(case, cfg):
    n, h, w, cin, cout, kh, kw, s, pad, relu, has_res = case
    ph, pw = (kh // 2, kw // 2) if pad else (0, 0)
    torch.manual_seed(0)
    x = _bf(torch.randn(n, cin, h, w))
    wt = _bf(torch.randn(cout, cin, kh, kw) * (2.0 / (cin * kh * kw)) ** 0.5)
    b = torch.randn(cout) * 0.1
    ref = F.conv2d(x, wt, b, stride=s, padding=(ph, pw))
    res = None
    if has_res:
        res = _bf(torch.randn_like(ref))
        ref = ref + res
    if relu:
        ref = F.relu(ref)
    wp, K, _ = ops.pack_weight(wt)
    xd = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    rd = res.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16) if res is not None else None
    y = ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), cout, kh, kw, (s, s), (ph, pw), relu=relu, residual=rd, cfg=cfg)
    torch.cuda.synchronize()
    got = y[..., :cout].float().cpu().permute(0, 3, 1, 2)
    assert got.shape == ref.shape
    assert _rel(got, ref) < 1.5e-2, _rel(got, ref)


def test_conv_stem_padded_input():
    """7x7/2 stem on a 3-channel image stored as 8 channels (zeros in 3..7)."""
    torch.manual_seed(1)
    x = _bf(torch.randn(2, 3, 40, 40))
    wt = _bf(torch.randn(64, 3, 7, 7) * 0.1)
    b = torch.randn(64) * 0.1
    ref = F.relu(F.conv2d(x, wt, b, stride=2, padding=3))
    x8 = torch.zeros(2, 40, 40, 8)
    x8[..., :3] = x.permute(0, 2, 3, 1)
    wp, K, _ = ops.pack_weight(wt, cin_eff=8)
    y = ops.conv2d_nhwc(x8.cuda().to(torch.bfloat16), wp.cuda(), b.cuda(), 64, 7, 7, (2, 2), (3, 3), relu=True)
    torch.cuda.synchronize()
    assert _rel(y.float().cpu().permute(0, 3, 1, 2), ref) < 1.5e-2


def test_conv_channel_offsets_concat():
    """Two convs writing disjoint channel ranges of one buffer + reading a slice."""
    torch.manual_seed(2)
    x = _bf(torch.randn(2, 96, 9, 9))
    w1 = _bf(torch.randn(32, 64, 1, 1) * 0.1)
    w2 = _bf(torch.randn(48, 32, 3, 3) * 0.1)
    b1, b2 = torch.randn(32) * 0.1, torch.randn(48) * 0.1
    xd = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    out = torch.full((2, 9, 9, 96), 7.0, device="cuda", dtype=torch.bfloat16)
    wp1, _, _ = ops.pack_weight(w1)
    wp2, _, _ = ops.pack_weight(w2)
    # conv1 reads channels [32:96) of x, writes channels [16:48) of out
    ops.conv2d_nhwc(xd, wp1.cuda(), b1.cuda(), 32, 1, 1, in_coff=32, cin=64, out=out, out_coff=16, relu=True)
    # conv2 reads channels [16:48) of out, writes channels [48:96) of out
    ops.conv2d_nhwc(out, wp2.cuda(), b2.cuda(), 48, 3, 3, pad=(1, 1), in_coff=16, cin=32, out=out, out_coff=48,
                    relu=True)
    torch.cuda.synchronize()
    r1 = F.relu(F.conv2d(x[:, 32:96], w1, b1))
    got = out.float().cpu().permute(0, 3, 1, 2)
    assert _rel(got[:, 16:48], r1) < 1.5e-2
    r2 = F.relu(F.conv2d(_bf(got[:, 16:48]), w2, b2, padding=1))
    assert _rel(got[:, 48:96], r2) < 1.5e-2
    assert torch.all(got[:, :16] == 7.0)


def test_fc_fp32_out():
    torch.manual_seed(3)
    x = _bf(torch.randn(5, 2048))
    wt = _bf(torch.randn(1000, 2048) * 0.02)
    b = torch.randn(1000) * 0.1
    ref = x @ wt.t() + b
    wp, K, _ = ops.pack_weight(wt[:, :, None, None])
    y = ops.conv2d_nhwc(x.view(5, 1, 1, 2048).cuda().to(torch.bfloat16), wp.cuda(), b.cuda(), 1000, 1, 1,
                        out_f32=True)
    torch.cuda.synchronize()
    assert _rel(y.view(5, -1)[:, :1000].cpu(), ref) < 5e-3


@pytest.mark.parametrize("ksplit,cfg", [(2, 14), (4, 11), (8, 14), (8, 23), (16, 22), (5, 15)])
def test_fc_split_k(ksplit, cfg):
    """Classifier GEMM with the K loop cut over workgroup slices: the fp32
    partial slices sum to x @ W^T + b (bias in slice 0 only), and the split
    softmax/top-5 over the slices equals softmax/top-5 of the summed logits."""
    torch.manual_seed(7)
    b_ = 37
    x = _bf(torch.randn(b_, 2048))
    wt = _bf(torch.randn(1000, 2048) * 0.02)
    b = torch.randn(1000) * 0.1
    ref = x @ wt.t() + b
    wp, K, _ = ops.pack_weight(wt[:, :, None, None])
    parts = ops.conv2d_nhwc(x.view(b_, 1, 1, 2048).cuda().to(torch.bfloat16), wp.cuda(), b.cuda(), 1000, 1, 1,
                            out_f32=True, cfg=cfg, ksplit=ksplit)
    torch.cuda.synchronize()
    assert parts.shape[0] == ksplit
    tot = parts.sum(0).view(b_, -1)[:, :1000].cpu()
    assert _rel(tot, ref) < 5e-3
    probs, idx, p = ops.softmax_top5(parts.view(ksplit, b_, -1)[..., :1000].contiguous())
    torch.cuda.synchronize()
    refp = torch.softmax(tot, -1)
    assert torch.allclose(probs.cpu(), refp, atol=1e-5, rtol=1e-3)
    assert torch.equal(idx.cpu().long(), refp.topk(5, dim=-1).indices)


@pytest.mark.parametrize("mode,k,s,pad", [("max", 3, 2, 0), ("max", 3, 2, 1), ("avg", 3, 1, 1)])
def test_pool(mode, k, s, pad):
    torch.manual_seed(4)
    x = _bf(torch.relu(torch.randn(2, 32, 17, 19)))
    if mode == "max":
        ref = F.max_pool2d(F.pad(x, (pad,) * 4), k, s)
    else:
        ref = F.avg_pool2d(x, k, s, padding=pad, count_include_pad=False)
    y = ops.pool3x3(x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16), mode, k, s, pad)
    torch.cuda.synchronize()
    assert _rel(y.float().cpu().permute(0, 3, 1, 2), ref) < 1e-2


@pytest.mark.parametrize("mode,k,s,pad,hw", [("max", 3, 2, 1, (9, 6)), ("max", 3, 1, 1, (5, 7)), ("max", 3, 2, 0, (71, 71)),
                                             ("avg", 3, 2, 1, (9, 6)), ("avg", 3, 1, 1, (1, 2)),
                                             ("max", 5, 2, 2, (9, 9)), ("avg", 5, 1, 2, (6, 5))])
def test_pool_signed(mode, k, s, pad, hw):
    """Signed inputs (padding must never win a max), edge windows, 1-pixel images; the
    k = 3 / pad <= 1 cases run the all-taps-in-flight kernel, k = 5 the generic one."""
    torch.manual_seed(5)
    x = _bf(torch.randn(3, 48, *hw))
    if mode == "max":
        ref = F.max_pool2d(F.pad(x, (pad,) * 4, value=float("-inf")), k, s)
    else:
        ref = F.avg_pool2d(x, k, s, padding=pad, count_include_pad=False)
    y = ops.pool3x3(x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16), mode, k, s, pad)
    torch.cuda.synchronize()
    got = y.float().cpu().permute(0, 3, 1, 2)
    assert got.shape == ref.shape
    assert _rel(got, ref) < 1e-2


@pytest.mark.parametrize("shape", [(3, 7, 7, 2048), (2, 8, 8, 2048), (5, 3, 5, 200), (1, 1, 1, 8)])
def test_global_avgpool(shape):
    x = _bf(torch.randn(*shape))
    y = ops.global_avgpool(x.cuda().to(torch.bfloat16))
    torch.cuda.synchronize()
    assert _rel(y.float().cpu(), x.mean(dim=(1, 2))) < 1e-2


def test_softmax_top5():
    torch.manual_seed(5)
    logits = torch.randn(37, 1000) * 3
    probs, idx, p = ops.softmax_top5(logits.cuda())
    torch.cuda.synchronize()
    ref = torch.softmax(logits, -1)
    assert torch.allclose(probs.cpu(), ref, atol=1e-6, rtol=1e-4)
    rv, ri = ref.topk(5, dim=-1)
    assert torch.equal(idx.cpu().long(), ri)
    assert torch.allclose(p.cpu(), rv, atol=1e-6, rtol=1e-4)


@pytest.mark.parametrize("rows,classes", [(5, 1000), (130, 1000), (3, 64), (9, 1024)])
def test_softmax_top5_ties_lower_id_first(rows, classes):
    """Coarse logits (many exact ties): top-5 ids in (value desc, id asc) order, the order the
    serving results have always used — the wave-per-row kernel keeps it."""
    torch.manual_seed(6)
    logits = torch.randint(-4, 5, (rows, classes)).float()
    probs, idx, p = ops.softmax_top5(logits.cuda())
    torch.cuda.synchronize()
    for r in range(rows):
        order = sorted(range(classes), key=lambda c: (-logits[r, c].item(), c))[:5]
        assert idx[r].cpu().tolist() == order, r
    ref = torch.softmax(logits, -1)
    assert torch.allclose(probs.cpu(), ref, atol=1e-6, rtol=1e-4)


@pytest.mark.parametrize("mode,hw", [("caffe", (224, 224)), ("tf", (299, 299))])
def test_preprocess(mode, hw):
    from distributed_machine_learning_amd.models.oracle import preprocess_reference

    torch.manual_seed(6)
    img = torch.randint(0, 256, (3, 300, 241, 3), dtype=torch.uint8)
    y = ops.preprocess(img.cuda(), hw, mode)
    torch.cuda.synchronize()
    ref = preprocess_reference(img, hw, mode)
    got = y.float().cpu().permute(0, 3, 1, 2)
    assert torch.all(got[:, 3:] == 0)
    assert (got[:, :3] - ref).abs().max().item() < 0.6  # bf16 rounding of values up to ~150


@pytest.mark.parametrize("kh,kw,s,p,hw,mode", [(7, 7, 2, 3, (224, 224), "caffe"), (3, 3, 2, 0, (299, 299), "tf")])
@pytest.mark.parametrize("cfg", [-1, 11, 15])
def test_pair_packed_stem(kh, kw, s, p, hw, mode, cfg):
    """preprocess(pair=True) + dilation-2 conv with pair-packed weights == the plain
    stem conv on the normal preprocess output."""
    from distributed_machine_learning_amd.models.engine import _r, pack_conv_weight, pair_pack_kernel
    from distributed_machine_learning_amd.models.oracle import preprocess_reference

    torch.manual_seed(7)
    img = torch.randint(0, 256, (2, hw[0], hw[1], 3), dtype=torch.uint8)
    k = torch.randn(kh, kw, 3, 64) * 0.05
    b = torch.randn(64) * 0.1
    x = _bf(preprocess_reference(img, hw, mode))
    ref = F.relu(F.conv2d(x, _bf(k.permute(3, 2, 0, 1)), b, stride=s, padding=p))
    xp = ops.preprocess(img.cuda(), hw, mode, pair=True, lpad=p)
    kp = pair_pack_kernel(k.numpy())
    K = kh * kp.shape[1] * 8
    wp = torch.from_numpy(pack_conv_weight(kp, 8, 256, _r(K, 64))).to(torch.bfloat16).cuda()
    y = ops.conv2d_nhwc(xp, wp, b.cuda(), 64, kh, kp.shape[1], (s, s), (p, 0), relu=True, dilation=(1, 2),
                        K=K, cfg=cfg, out_hw=tuple(ref.shape[2:]))
    torch.cuda.synchronize()
    got = y.float().cpu().permute(0, 3, 1, 2)
    assert _rel(got, ref) < 1.5e-2, _rel(got, ref)


@pytest.mark.parametrize("cfg", [-1, 11, 14, 15])
@pytest.mark.parametrize("stride", [1, 2])
def test_fused_sibling_1x1_segments(cfg, stride):
    """One segmented GEMM == three separate 1x1 convs writing to a concat buffer
    at offsets and to a temporary (Inception mixed-block / ResNet stage-entry fusion)."""
    torch.manual_seed(8)
    x = _bf(torch.randn(2, 96, 13, 11))
    specs = [(64, True), (48, False), (32, True)]
    ws = [_bf(torch.randn(co, 96, 1, 1) * 0.1) for co, _ in specs]
    bs = [torch.randn(co) * 0.1 for co, _ in specs]
    ho, wo = (13 - 1) // stride + 1, (11 - 1) // stride + 1
    concat = torch.full((2, ho, wo, 160), 3.0, device="cuda", dtype=torch.bfloat16)
    tmp = torch.zeros((2, ho, wo, 48), device="cuda", dtype=torch.bfloat16)
    xd = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    ops.fused_conv1x1(xd, [(ws[0], bs[0], concat, 0, True), (ws[1], bs[1], tmp, 0, False),
                           (ws[2], bs[2], concat, 96, True)], stride=stride, cfg=cfg)
    refs = [F.conv2d(x, w, b, stride=stride) for w, b in zip(ws, bs)]
    got = concat.float().cpu().permute(0, 3, 1, 2)
    assert _rel(got[:, 0:64], F.relu(refs[0])) < 1.5e-2
    assert _rel(tmp.float().cpu().permute(0, 3, 1, 2), refs[1]) < 1.5e-2
    assert _rel(got[:, 96:128], F.relu(refs[2])) < 1.5e-2
    assert torch.all(got[:, 64:96] == 3.0) and torch.all(got[:, 128:] == 3.0)


def test_avgpool_relu_flag():
    torch.manual_seed(9)
    x = _bf(torch.randn(2, 16, 9, 9))
    y = ops.pool3x3(x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16), "avg", 3, 1, 1, relu=True)
    torch.cuda.synchronize()
    ref = F.relu(F.avg_pool2d(x, 3, 1, padding=1, count_include_pad=False))
    assert _rel(y.float().cpu().permute(0, 3, 1, 2), ref) < 1e-2


@pytest.mark.parametrize("cfg", [10, 11, 12, 13, 14, 15, 16, 17, 18, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33,
                                 34, 36, 37, 38, 39, 48, 49, 56, 57, 58, 59, 60])
@pytest.mark.parametrize("case", [(2, 28, 28, 64, 256, 1, 1), (2, 14, 10, 128, 512, 1, 1), (2, 7, 9, 64, 64, 3, 3)])
def test_conv_subsampled_residual(case, cfg):
    """Residual read at stride 2 from its full-resolution grid (rsub = 2: the
    epilogue of a block whose stride-2 consumer was pushed up, models/optimize.py)."""
    n, ho, wo, cin, cout, kh, kw = case
    torch.manual_seed(1)
    x = _bf(torch.randn(n, cin, ho, wo))
    wt = _bf(torch.randn(cout, cin, kh, kw) * (2.0 / (cin * kh * kw)) ** 0.5)
    b = torch.randn(cout) * 0.1
    res = _bf(torch.randn(n, cout, 2 * ho, 2 * wo))
    ref = F.relu(F.conv2d(x, wt, b, padding=(kh // 2, kw // 2)) + res[:, :, ::2, ::2])
    wp, K, _ = ops.pack_weight(wt)
    xd = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    rd = res.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    y = ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), cout, kh, kw, (1, 1), (kh // 2, kw // 2), relu=True, residual=rd,
                        cfg=cfg)
    torch.cuda.synchronize()
    got = y[..., :cout].float().cpu().permute(0, 3, 1, 2)
    assert _rel(got, ref) < 1.5e-2, _rel(got, ref)


def test_conv_non_tile_config_refused():
    """cfg ids outside the v2 tile configs (the removed v1 / halo kernels) and
    shapes no tile config can run fail loudly on the host."""
    x = torch.zeros(1, 4, 4, 64, device="cuda", dtype=torch.bfloat16)
    wp, _, _ = ops.pack_weight(torch.zeros(64, 64, 1, 1))
    for cfg in (0, 4, 35, 40, 64):
        with pytest.raises(Exception):
            ops.conv2d_nhwc(x, wp.cuda(), torch.zeros(64), 64, 1, 1, cfg=cfg)


GROUP_CASES = [
    # n, h, w, members: (cin, in_coff, cout, kh, kw, stride) — all write one concat buffer
    (2, 17, 17, [(128, 0, 192, 1, 7, 1), (96, 128, 64, 7, 1, 1)]),
    (1, 35, 35, [(48, 0, 64, 5, 5, 1), (64, 48, 96, 3, 3, 1)]),
    (2, 8, 8, [(384, 0, 384, 1, 3, 1), (384, 0, 384, 3, 1, 1), (448, 384, 384, 3, 3, 1), (64, 832, 64, 1, 1, 1)]),
    (2, 17, 17, [(160, 0, 320, 3, 3, 2), (128, 160, 192, 3, 3, 2)]),
]


@pytest.mark.parametrize("case", GROUP_CASES)
@pytest.mark.parametrize("cfg", [11, 12, 14, 15, 17, 22, 23, 24, 25, 26, 27, 28, 29, 32, 33])
def test_conv_group_matches_members(case, cfg):
    """dml_conv_group: independent convs (different kh x kw / Cin / Cout, input
    channel slices of one tensor, outputs at channel offsets of one concat
    buffer) in ONE grid == each conv launched alone on the same tile config
    (bit-exact), and == the fp32 reference; channels nobody writes stay put."""
    n, h, w, members = case
    torch.manual_seed(3)
    ctot = max(c0 + ci for ci, c0, *_ in members)
    x = _bf(torch.randn(n, ctot, h, w))
    xd = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    s = members[0][5]
    ho, wo = (h + s - 1) // s if s == 1 else (h - 3) // s + 1, (w + s - 1) // s if s == 1 else (w - 3) // s + 1
    cout_tot = sum(m[2] for m in members) + 8
    outs = [torch.full((n, ho, wo, cout_tot), 7.0, device="cuda", dtype=torch.bfloat16) for _ in range(2)]
    refs, deferred, keep = [], [], []
    for (ci, c0, co, kh, kw, st) in members:
        wt = _bf(torch.randn(co, ci, kh, kw) * (2.0 / (ci * kh * kw)) ** 0.5)
        b = torch.randn(co) * 0.1
        pad = (kh // 2, kw // 2) if st == 1 else (0, 0)
        refs.append(F.relu(F.conv2d(x[:, c0:c0 + ci], wt, b, stride=st, padding=pad)))
        wp = ops.pack_weight(wt)[0].cuda()
        keep.append(wp)
        off = sum(r.shape[1] for r in refs[:-1])
        common = dict(stride=(st, st), pad=pad, relu=True, in_coff=c0, cin=ci, out_coff=off)
        ops.conv2d_nhwc(xd, wp, b.cuda(), co, kh, kw, out=outs[0], cfg=cfg, **common)
        y = ops.conv2d_nhwc(xd, wp, b.cuda(), co, kh, kw, out=outs[1], defer=deferred, **common)
        keep.append(y._keep)
    ops.conv_group(deferred, cfg)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    got = outs[1].float().cpu().permute(0, 3, 1, 2)
    off = 0
    for r in refs:
        assert _rel(got[:, off:off + r.shape[1]], r) < 1.5e-2
        off += r.shape[1]
    assert torch.all(got[:, off:] == 7.0)


def test_conv_group_refuses_bad_members():
    x = torch.zeros(1, 8, 8, 64, device="cuda", dtype=torch.bfloat16)
    wp = ops.pack_weight(torch.zeros(64, 64, 1, 1))[0].cuda()
    d = []
    ops.conv2d_nhwc(x, wp, torch.zeros(64), 64, 1, 1, defer=d)
    ops.conv2d_nhwc(x, wp, torch.zeros(64), 64, 1, 1, residual=x, defer=d)
    from distributed_machine_learning_amd import _native as N
    with pytest.raises(N.NativeError, match="residual-free"):
        ops.conv_group(d, 14)
    with pytest.raises(N.NativeError, match="grouped"):
        ops.conv_group(d[:1], 10)


@pytest.mark.parametrize("cfg", [11, 14, 22, 29])
def test_conv_group_with_pools(cfg):
    """A grouped grid holding convs AND 3x3 pools (an Inception level: 5x5 + 3x3
    branch convs + the pool branch's avg pool; a reduction block's 3x3/2 conv +
    max pool) == the same ops launched one by one, bit-exact."""
    torch.manual_seed(4)
    n, h, w = 2, 17, 17
    x = _bf(torch.randn(n, 64, h, w)).permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    pin = _bf(torch.randn(n, 32, h, w)).permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    wts = [(_bf(torch.randn(96, 64, k, k) * 0.05), k) for k in (5, 3)]
    wps = [(ops.pack_weight(wt)[0].cuda(), k) for wt, k in wts]
    b = torch.randn(96).cuda() * 0.1
    outs = [torch.full((n, h, w, 96 * 2 + 32 + 8), 3.0, device="cuda", dtype=torch.bfloat16) for _ in range(2)]
    mp = [torch.zeros(n, 8, 8, 64, device="cuda", dtype=torch.bfloat16) for _ in range(2)]
    d, dp = [], []
    for o, (wp, k) in zip((0, 96), wps):
        ops.conv2d_nhwc(x, wp, b, 96, k, k, pad=(k // 2, k // 2), relu=True, out=outs[0], out_coff=o, cfg=cfg)
        ops.conv2d_nhwc(x, wp, b, 96, k, k, pad=(k // 2, k // 2), relu=True, out=outs[1], out_coff=o, defer=d)
    ops.pool3x3(pin, "avg", stride=1, pad=1, out=outs[0], out_coff=192, relu=True)
    ops.pool3x3(pin, "avg", stride=1, pad=1, out=outs[1], out_coff=192, relu=True, defer=dp)
    ops.pool3x3(x, "max", stride=2, pad=0, out=mp[0])
    ops.pool3x3(x, "max", stride=2, pad=0, out=mp[1], defer=dp)
    ops.conv_group(d, cfg, dp)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(mp[0], mp[1])
    ref = F.avg_pool2d(pin.float().permute(0, 3, 1, 2), 3, 1, 1, count_include_pad=False).relu()
    assert _rel(outs[1][..., 192:224].float().permute(0, 3, 1, 2).cpu(), ref.cpu()) < 1e-2
    assert torch.all(outs[1][..., 224:] == 3.0)
    from distributed_machine_learning_amd import _native as N
    bad = list(dp)
    bad[0].k = 5
    with pytest.raises(N.NativeError, match="pool members"):
        ops.conv_group(d, cfg, bad)

