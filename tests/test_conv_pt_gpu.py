"""Patch-stationary stride-1 conv tiles (csrc/kernels/conv_igemm_pt.hip, cfg 140..): numerics
against a plain-PyTorch fp32 conv of the same bf16 inputs (the K order is chunk-major, so not
bit-identical to the v2 tiles), on the stride-1 layer classes of both networks — row-block
tiles with a partial last block, multi-image tiles with a partial last tile, 1x7 / 7x1 / 1x3 /
3x1 / 5x5 / 'valid', residual, subsampled residual, channel offsets — and the refusals (stride 2, Cin % 64, a patch larger than the config's)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from distributed_machine_learning_amd import _native as N, ops  # noqa: E402
from distributed_machine_learning_amd.ops import tuning  # noqa: E402

from test_kernels_gpu import _bf, _rel  # noqa: E402

PT = list(tuning.PT_CFGS)
CASES = [
    # n, h, w, cin, cout, kh, kw, pad, relu, residual
    (3, 14, 14, 128, 128, 3, 3, True, True, False),    # one image per 256-px tile
    (11, 7, 7, 64, 64, 3, 3, True, True, True),        # 5 images per tile, partial last tile, residual
    (2, 23, 19, 64, 192, 3, 3, True, True, False),     # row blocks, partial last block, 2 channel tiles
    (2, 17, 17, 128, 192, 1, 7, True, True, False),    # 1x7 'same'
    (2, 17, 17, 128, 160, 7, 1, True, False, False),   # 7x1 'same', no ReLU
    (3, 8, 8, 384, 384, 1, 3, True, True, False),      # 1x3 on 8x8
    (3, 8, 8, 448, 384, 3, 3, True, True, False),      # 3x3 on 8x8, 7 chunks
    (2, 12, 12, 64, 96, 5, 5, True, True, False),      # 5x5 'same'
    (2, 13, 11, 64, 64, 3, 3, False, True, False),     # 'valid'
    (2, 56, 56, 64, 64, 3, 3, True, True, False),      # ResNet50 stage 2 geometry
]


def _ref(case):
    n, h, w, cin, cout, kh, kw, pad, relu, has_res = case
    ph, pw = (kh // 2, kw // 2) if pad else (0, 0)
    torch.manual_seed(0)
    x = _bf(torch.randn(n, cin, h, w))
    wt = _bf(torch.randn(cout, cin, kh, kw) * (2.0 / (cin * kh * kw)) ** 0.5)
    b = torch.randn(cout) * 0.1
    ref = F.conv2d(x, wt, b, padding=(ph, pw))
    res = _bf(torch.randn_like(ref)) if has_res else None
    if res is not None:
        ref = ref + res
    if relu:
        ref = F.relu(ref)
    return x, wt, b, res, ref, (ph, pw)


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("cfg", PT)
def test_pt_conv_matches_fp32(case, cfg):
    x, wt, b, res, ref, (ph, pw) = _ref(case)
    n, h, w, cin, cout, kh, kw, pad, relu, has_res = case
    wp, K, _ = ops.pack_weight(wt)
    xd = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    rd = res.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16) if res is not None else None
    try:
        y = ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), cout, kh, kw, (1, 1), (ph, pw), relu=relu, residual=rd, cfg=cfg)
    except N.NativeError as e:
        assert "dml_conv_pt" in str(e)
        pytest.skip(f"cfg {cfg} refuses this shape (its patch does not fit): {e}")
    torch.cuda.synchronize()
    got = y[..., :cout].float().cpu().permute(0, 3, 1, 2)
    assert _rel(got, ref) < 1.5e-2, _rel(got, ref)


def test_pt_covers_the_target_layers():
    """The 256-pixel configs take every ResNet50 3x3 and the InceptionV3 stride-1 shapes with
    Cin % 64 == 0 (a refusal here would silently leave a layer on the other tiles)."""
    for case in [(2, 14, 14, 256, 256, 3, 3, True, True, False), (2, 7, 7, 512, 512, 3, 3, True, True, False),
                 (2, 28, 28, 128, 128, 3, 3, True, True, False), (2, 56, 56, 64, 64, 3, 3, True, True, False),
                 (2, 17, 17, 192, 192, 1, 7, True, True, False), (2, 8, 8, 384, 384, 3, 1, True, True, False)]:
        x, wt, b, res, ref, (ph, pw) = _ref(case)
        wp, K, _ = ops.pack_weight(wt)
        xd = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
        y = ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), case[4], case[5], case[6], (1, 1), (ph, pw), relu=True, cfg=140)
        torch.cuda.synchronize()
        assert _rel(y[..., :case[4]].float().cpu().permute(0, 3, 1, 2), ref) < 1.5e-2


@pytest.mark.parametrize("cfg", PT)
def test_pt_subsampled_residual_and_channel_offsets(cfg):
    """Output into a channel slice of a wider buffer, input from a channel slice, residual read
    at stride 2 from its full-resolution grid (the pushed-down ResNet shortcut)."""
    torch.manual_seed(3)
    n, ho, wo, cin, cout = 2, 14, 10, 64, 128
    xfull = _bf(torch.randn(n, cin + 64, ho, wo))
    x = xfull[:, 64:]
    wt = _bf(torch.randn(cout, cin, 3, 3) * (2.0 / (cin * 9)) ** 0.5)
    b = torch.randn(cout) * 0.1
    res = _bf(torch.randn(n, cout, 2 * ho, 2 * wo))
    ref = F.relu(F.conv2d(x, wt, b, padding=1) + res[:, :, ::2, ::2])
    wp, K, _ = ops.pack_weight(wt)
    xd = xfull.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    rd = res.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    out = torch.full((n, ho, wo, cout + 32), 7.0, device="cuda", dtype=torch.bfloat16)
    try:
        ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), cout, 3, 3, (1, 1), (1, 1), relu=True, residual=rd, out=out,
                        out_coff=32, in_coff=64, cin=cin, cfg=cfg)
    except N.NativeError:
        pytest.skip("refused")
    torch.cuda.synchronize()
    got = out[..., 32:].float().cpu().permute(0, 3, 1, 2)
    assert _rel(got, ref) < 1.5e-2
    assert torch.all(out[..., :32] == 7.0)


@pytest.mark.parametrize("bad", ["stride2", "cin80", "ksplit"])
def test_pt_refusals(bad):
    x = torch.zeros(2, 16, 16, 80 if bad == "cin80" else 64, device="cuda", dtype=torch.bfloat16)
    wp, _, _ = ops.pack_weight(torch.zeros(64, x.shape[-1], 3, 3))
    with pytest.raises(N.NativeError):
        ops.conv2d_nhwc(x, wp.cuda(), torch.zeros(64).cuda(), 64, 3, 3, (2, 2) if bad == "stride2" else (1, 1),
                        (1, 1), cfg=140, ksplit=2 if bad == "ksplit" else 1, out_f32=bad == "ksplit")
