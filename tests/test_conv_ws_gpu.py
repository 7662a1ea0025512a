"""Warp-specialised implicit-GEMM conv tiles (csrc/kernels/conv_igemm_ws.hip, cfg 100..; the
persistent form, conv_igemm_wsp.hip, cfg 120..):
numerics against a plain-PyTorch fp32 conv of the same bf16 inputs, and BIT-identical to a
v2 tile (conv_igemm_v2.hip) — both accumulate every output element over K in the same
MFMA k-step order, so only the work split between waves differs. Covers every conv class
of SURVEY §2.7 (1x1 s1/s2, 3x3, 5x5, 1x7 / 7x1 / 1x3 / 3x1, tap-straddling Cin 80, residual,
subsampled residual, segmented sibling outputs, fp32 split-K)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from distributed_machine_learning_amd import ops  # noqa: E402
from distributed_machine_learning_amd.ops import tuning  # noqa: E402

from test_kernels_gpu import CONV_CASES, _bf, _rel  # noqa: E402

WS = list(tuning.WS_CFGS) + list(tuning.WSP_CFGS)  # per-tile and persistent forms


def _conv_case(case):
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

    def run(cfg):
        y = ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), cout, kh, kw, (s, s), (ph, pw), relu=relu, residual=rd, cfg=cfg)
        torch.cuda.synchronize()
        return y
    return run, ref, cout


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("cfg", WS)
def test_ws_conv_matches_fp32_and_v2(case, cfg):
    run, ref, cout = _conv_case(case)
    y = run(cfg)
    got = y[..., :cout].float().cpu().permute(0, 3, 1, 2)
    assert _rel(got, ref) < 1.5e-2, _rel(got, ref)
    assert torch.equal(y, run(11)), "warp-specialised tile differs from the v2 tile"


@pytest.mark.parametrize("cfg", WS)
@pytest.mark.parametrize("case", [(2, 28, 28, 64, 256, 1, 1), (2, 14, 10, 128, 512, 1, 1), (2, 7, 9, 64, 64, 3, 3)])
def test_ws_subsampled_residual(case, cfg):
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


@pytest.mark.parametrize("cfg", WS)
def test_ws_fused_sibling_segments(cfg):
    torch.manual_seed(8)
    x = _bf(torch.randn(2, 96, 13, 11))
    specs = [(64, True), (48, False), (32, True)]
    ws = [_bf(torch.randn(co, 96, 1, 1) * 0.1) for co, _ in specs]
    bs = [torch.randn(co) * 0.1 for co, _ in specs]
    concat = torch.full((2, 13, 11, 160), 3.0, device="cuda", dtype=torch.bfloat16)
    tmp = torch.zeros((2, 13, 11, 48), device="cuda", dtype=torch.bfloat16)
    xd = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    ops.fused_conv1x1(xd, [(ws[0], bs[0], concat, 0, True), (ws[1], bs[1], tmp, 0, False),
                           (ws[2], bs[2], concat, 96, True)], cfg=cfg)
    refs = [F.conv2d(x, w, b) for w, b in zip(ws, bs)]
    got = concat.float().cpu().permute(0, 3, 1, 2)
    assert _rel(got[:, 0:64], F.relu(refs[0])) < 1.5e-2
    assert _rel(tmp.float().cpu().permute(0, 3, 1, 2), refs[1]) < 1.5e-2
    assert _rel(got[:, 96:128], F.relu(refs[2])) < 1.5e-2
    assert torch.all(got[:, 64:96] == 3.0) and torch.all(got[:, 128:] == 3.0)


def test_wsp_refuses_split_k():
    x = torch.zeros(4, 1, 1, 2048, device="cuda", dtype=torch.bfloat16)
    wp, _, _ = ops.pack_weight(torch.zeros(1000, 2048, 1, 1))
    with pytest.raises(Exception):
        ops.conv2d_nhwc(x, wp.cuda(), torch.zeros(1000), 1000, 1, 1, out_f32=True, cfg=120, ksplit=2)


def test_wsp_many_tiles_per_workgroup():
    """A conv with far more tiles than resident workgroups (each persistent workgroup runs a
    long tile list through one ring) and an M tail, bit-identical to the v2 tile."""
    run, ref, cout = _conv_case((9, 57, 57, 64, 64, 3, 3, 1, 1, True, False))
    for cfg in tuning.WSP_CFGS:
        assert torch.equal(run(cfg), run(15)), cfg


@pytest.mark.parametrize("ksplit,cfg", [(2, 100), (4, 104), (8, 110), (5, 103)])
def test_ws_fc_split_k(ksplit, cfg):
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
    tot = parts.sum(0).view(b_, -1)[:, :1000].cpu()
    assert _rel(tot, ref) < 5e-3
