"""Numerics of the Winograd F(2x2, 3x3) kernel (csrc/kernels/conv_wino.hip,
cfg 80) against a plain-PyTorch fp32 conv of the same bf16-rounded inputs, on
every stride-1 3x3 shape class of ResNet50 / InceptionV3 (same and valid
padding, Cin % 32 != 0, Cout % 64 != 0, odd spatial sizes, channel-offset input
and output) — held to the implicit GEMM's bound (1.5e-2) — and against the CPU
model of its arithmetic (ops/winograd.conv_model) much more tightly."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from distributed_machine_learning_amd import ops  # noqa: E402
from distributed_machine_learning_amd.ops import winograd as W  # noqa: E402


def _bf(x):
    return x.to(torch.bfloat16).float()


def _rel(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


CASES = [  # n, h, w, cin, cout, pad, relu
    (4, 56, 56, 64, 64, 1, True),      # ResNet50 stage 2
    (2, 28, 28, 128, 128, 1, True),    # stage 3
    (4, 14, 14, 256, 256, 1, True),    # stage 4
    (8, 7, 7, 512, 512, 1, True),      # stage 5 (odd size: half-empty edge tiles)
    (2, 35, 35, 64, 96, 1, True),      # InceptionV3 mixed 3x3 (Cout % 64 != 0)
    (2, 35, 35, 96, 96, 1, False),
    (1, 73, 73, 80, 192, 0, True),     # conv2d_5: valid, Cin % 32 != 0
    (3, 8, 8, 448, 384, 1, True),      # mixed9/10 3x3
    (2, 9, 11, 40, 72, 1, True),       # ragged everything
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("cfg", [80, 81, 82, 83])
def test_wino_matches_fp32(case, cfg):
    n, h, w, cin, cout, pad, relu = case
    torch.manual_seed(hash(case) % 1000)
    x = _bf(torch.randn(n, cin, h, w))
    wt = _bf(torch.randn(cout, cin, 3, 3) * (2.0 / (cin * 9)) ** 0.5)
    b = torch.randn(cout) * 0.1
    ref = F.conv2d(x, wt, b, padding=pad)
    if relu:
        ref = F.relu(ref)
    wp, K, _ = ops.pack_weight(wt)
    wu = ops.pack_wino_weight(wt).cuda()
    xd = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    try:
        y = ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), cout, 3, 3, (1, 1), (pad, pad), relu=relu, cfg=cfg, wu=wu)
    except ops.N.NativeError as e:  # a patch config whose LDS patch is too small for this shape
        assert cfg == 82 and "patch" in str(e), e
        pytest.skip(str(e))
    torch.cuda.synchronize()
    got = y[..., :cout].float().cpu()
    assert _rel(got.permute(0, 3, 1, 2), ref) < 1.5e-2, _rel(got.permute(0, 3, 1, 2), ref)
    # the kernel's own arithmetic (bf16 V and U, fp32 sums) modelled on the CPU
    u = W._bf16(W.filter_transform(wt.permute(2, 3, 1, 0).numpy()))
    model = W.conv_model(x.permute(0, 2, 3, 1).numpy(), u, b.numpy(), pad, relu)
    assert _rel(got, torch.from_numpy(model)) < 4e-3, _rel(got, torch.from_numpy(model))
    # the same conv on the implicit GEMM (cfg 15) agrees within both kernels' error
    y2 = ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), cout, 3, 3, (1, 1), (pad, pad), relu=relu, cfg=15)
    torch.cuda.synchronize()
    assert _rel(got, y2[..., :cout].float().cpu()) < 2e-2


@pytest.mark.parametrize("cfg", [80, 81, 82, 83])
def test_wino_channel_offsets(cfg):
    """Input read from a channel slice of a wider buffer, output written at a channel
    offset of a concat buffer (InceptionV3's branch layout); nothing else is touched."""
    torch.manual_seed(5)
    n, h, w, cin, cout = 2, 17, 17, 96, 64
    buf = _bf(torch.randn(n, h, w, 160)).cuda().to(torch.bfloat16)
    x = buf[..., 32:32 + cin].float().cpu().permute(0, 3, 1, 2)
    wt = _bf(torch.randn(cout, cin, 3, 3) * 0.05)
    b = torch.randn(cout) * 0.1
    ref = F.relu(F.conv2d(x, wt, b, padding=1)).permute(0, 2, 3, 1)
    out = torch.full((n, h, w, 192), 7.0, device="cuda", dtype=torch.bfloat16)
    wp, _, _ = ops.pack_weight(wt)
    ops.conv2d_nhwc(buf, wp.cuda(), b.cuda(), cout, 3, 3, (1, 1), (1, 1), relu=True, out=out, out_coff=64,
                    in_coff=32, cin=cin, cfg=cfg, wu=ops.pack_wino_weight(wt).cuda())
    torch.cuda.synchronize()
    o = out.float().cpu()
    assert _rel(o[..., 64:128], ref) < 1.5e-2
    assert (o[..., :64] == 7.0).all() and (o[..., 128:] == 7.0).all()


def test_wino_refuses_what_it_cannot_run():
    from distributed_machine_learning_amd._native import NativeError

    x = torch.zeros(1, 8, 8, 64, device="cuda", dtype=torch.bfloat16)
    wt = torch.zeros(64, 64, 3, 3)
    wp, _, _ = ops.pack_weight(wt)
    with pytest.raises(NativeError):  # stride 2
        ops.conv2d_nhwc(x, wp.cuda(), torch.zeros(64).cuda(), 64, 3, 3, (2, 2), (1, 1), cfg=ops.WINO_CFG,
                        wu=ops.pack_wino_weight(wt).cuda())
    with pytest.raises(NativeError):  # no transformed weights
        ops.conv2d_nhwc(x, wp.cuda(), torch.zeros(64).cuda(), 64, 3, 3, (1, 1), (1, 1), cfg=ops.WINO_CFG)
