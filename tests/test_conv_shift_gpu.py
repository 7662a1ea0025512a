"""Numerics of the shifted-pixel stride-1 conv kernel (csrc/kernels/conv_shift.hip,
cfg ids 64..) against a plain-PyTorch fp32 conv of the same bf16-rounded
operands, on every shape class it serves: ResNet50's 3x3 stages (one and
several channel chunks, 56x56 halos of 370 rows, 7x7 images several per tile,
M tails), InceptionV3's 1x7 / 7x1 / 1x3 / 3x1 and 3x3 at 35x35 (Cout tails
inside a channel tile), residual + ReLU epilogues, input/output channel
offsets; shapes it cannot serve are refused on the host."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from distributed_machine_learning_amd import ops  # noqa: E402

SHIFT_CFGS = [64, 65, 66, 67, 68, 69]
CASES = [
    # n, h, w, cin, cout, kh, kw, relu, residual
    (2, 14, 14, 64, 64, 3, 3, True, False),
    (2, 28, 28, 128, 128, 3, 3, True, True),
    (3, 7, 7, 512, 512, 3, 3, True, False),
    (2, 56, 56, 64, 64, 3, 3, True, False),
    (1, 17, 17, 128, 192, 1, 7, True, False),
    (1, 17, 17, 128, 192, 7, 1, False, False),
    (2, 8, 8, 384, 384, 1, 3, True, False),
    (2, 8, 8, 384, 384, 3, 1, True, True),
    (1, 35, 35, 64, 96, 3, 3, True, False),
    (5, 13, 11, 192, 64, 3, 3, False, True),
]


def _bf(x):
    return x.to(torch.bfloat16).float()


def _rel(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


def _case(case, seed=0):
    n, h, w, cin, cout, kh, kw, relu, has_res = case
    torch.manual_seed(seed)
    x = _bf(torch.randn(n, cin, h, w))
    wt = _bf(torch.randn(cout, cin, kh, kw) * (2.0 / (cin * kh * kw)) ** 0.5)
    b = torch.randn(cout) * 0.1
    ref = F.conv2d(x, wt, b, padding=(kh // 2, kw // 2))
    res = _bf(torch.randn_like(ref)) if has_res else None
    if res is not None:
        ref = ref + res
    if relu:
        ref = F.relu(ref)
    return x, wt, b, res, ref


def _fits(case, cfg):
    n, h, w, cin, cout, kh, kw, _, _ = case
    bm = 256 if cfg in (64, 65, 68) else 128
    halo = 384 if bm == 256 else 256
    bk = 64 if cfg in (64, 67, 68) else 32
    return cin % bk == 0 and bm + 2 * ((kh // 2) * w + kw // 2) <= halo


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("cfg", SHIFT_CFGS)
def test_conv_shift_matches_fp32(case, cfg):
    if not _fits(case, cfg):
        pytest.skip("shape outside this config's halo / channel chunk (refusal tested below)")
    n, h, w, cin, cout, kh, kw, relu, _ = case
    x, wt, b, res, ref = _case(case)
    wp, _, _ = ops.pack_weight(wt)
    xd = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    rd = res.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16) if res is not None else None
    y = ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), cout, kh, kw, (1, 1), (kh // 2, kw // 2), relu=relu, residual=rd,
                        cfg=cfg)
    y2 = ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), cout, kh, kw, (1, 1), (kh // 2, kw // 2), relu=relu, residual=rd,
                         cfg=11)
    torch.cuda.synchronize()
    got = y[..., :cout].float().cpu().permute(0, 3, 1, 2)
    assert got.shape == ref.shape
    assert _rel(got, ref) < 1.5e-2, _rel(got, ref)
    # same bf16 operands, fp32 accumulation in another order: within bf16 output rounding of the implicit GEMM
    assert _rel(got, y2[..., :cout].float().cpu().permute(0, 3, 1, 2)) < 1e-2


@pytest.mark.parametrize("cfg", [64, 66])
def test_conv_shift_channel_offsets(cfg):
    """Reads channels [64:192) of a 256-wide buffer, writes channels [32:160) of
    a 224-wide buffer (ldx, ldy != Cin, Cout); the rest of the output untouched."""
    torch.manual_seed(5)
    x = _bf(torch.randn(2, 256, 15, 15))
    wt = _bf(torch.randn(128, 128, 3, 3) * 0.05)
    b = torch.randn(128) * 0.1
    wp, _, _ = ops.pack_weight(wt)
    xd = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    out = torch.full((2, 15, 15, 224), 3.0, device="cuda", dtype=torch.bfloat16)
    ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), 128, 3, 3, pad=(1, 1), in_coff=64, cin=128, out=out, out_coff=32,
                    relu=True, cfg=cfg)
    torch.cuda.synchronize()
    ref = F.relu(F.conv2d(x[:, 64:192], wt, b, padding=1))
    got = out.float().cpu().permute(0, 3, 1, 2)
    assert _rel(got[:, 32:160], ref) < 1.5e-2
    assert torch.all(got[:, :32] == 3.0) and torch.all(got[:, 160:] == 3.0)


def test_conv_shift_refuses_unsupported():
    x = torch.zeros(1, 35, 35, 48, device="cuda", dtype=torch.bfloat16)
    w5, _, _ = ops.pack_weight(torch.zeros(64, 48, 5, 5))
    with pytest.raises(Exception):   # Cin 48 % BK and a 400-row halo
        ops.conv2d_nhwc(x, w5.cuda(), torch.zeros(64), 64, 5, 5, pad=(2, 2), cfg=64)
    x = torch.zeros(1, 14, 14, 64, device="cuda", dtype=torch.bfloat16)
    w3, _, _ = ops.pack_weight(torch.zeros(64, 64, 3, 3))
    with pytest.raises(Exception):   # stride 2
        ops.conv2d_nhwc(x, w3.cuda(), torch.zeros(64), 64, 3, 3, (2, 2), (1, 1), cfg=66)
    with pytest.raises(Exception):   # valid padding
        ops.conv2d_nhwc(x, w3.cuda(), torch.zeros(64), 64, 3, 3, (1, 1), (0, 0), cfg=66)
