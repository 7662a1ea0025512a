"""Generic row-ring conv family (csrc/kernels/conv_rowring.hip, cfg 160..177) on the GPU:
numerics of every config the launcher accepts against a plain-PyTorch fp32 conv of the same
bf16 inputs on the InceptionV3 / ResNet50 stride-1 classes (3x3 'valid' Cin 80, 3x3 / 5x5
'same', 1x7 / 7x1, 1x3 / 3x1, ResNet50 stage 3), channel-offset input and output, and the
refusals. The index math is modelled on the CPU (tests/test_conv_rrg_model.py)."""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from distributed_machine_learning_amd import _native as N, ops  # noqa: E402
from distributed_machine_learning_amd.ops import tuning  # noqa: E402

from test_kernels_gpu import _bf, _rel  # noqa: E402

CASES = [  # n, h, w, cin, cout, kh, kw, same, relu
    (2, 73, 73, 80, 192, 3, 3, False, True),    # InceptionV3 conv2d_5
    (3, 35, 35, 64, 96, 3, 3, True, True),      # mixed 3x3 64 -> 96
    (2, 35, 35, 96, 96, 3, 3, True, False),     # 96 -> 96, no ReLU
    (2, 35, 35, 48, 64, 5, 5, True, True),      # 5x5
    (2, 17, 17, 160, 160, 1, 7, True, True),    # 1x7
    (2, 17, 17, 160, 192, 7, 1, True, True),    # 7x1
    (2, 8, 8, 384, 384, 1, 3, True, True),      # 1x3
    (1, 28, 28, 128, 128, 3, 3, True, True),    # ResNet50 stage 3
    (1, 56, 56, 64, 64, 3, 3, True, True),      # ResNet50 stage 2
]


def _args(x, wp, b, y, cin, ldx, cout, kh, kw, ph, pw, relu=True):
    n, h, w = x.shape[:3]
    return N.ConvArgs(x.data_ptr(), wp.data_ptr(), b.data_ptr(), None, y.data_ptr(), n, h, w, cin, ldx, kh, kw, 1, 1,
                      ph, pw, h + 2 * ph - kh + 1, w + 2 * pw - kw + 1, cout, kh * kw * cin, wp.shape[1], y.shape[-1],
                      0, int(relu), 0, 1, 1)


@pytest.mark.parametrize("case", CASES)
def test_rrg_matches_fp32(case):
    n, h, w, cin, cout, kh, kw, same, relu = case
    torch.manual_seed(1)
    ph, pw = ((kh - 1) // 2, (kw - 1) // 2) if same else (0, 0)
    x = _bf(torch.randn(n, cin, h, w))
    wt = _bf(torch.randn(cout, cin, kh, kw) * (2.0 / (cin * kh * kw)) ** 0.5)
    b = torch.randn(cout) * 0.1
    ref = F.conv2d(x, wt, b, padding=(ph, pw))
    if relu:
        ref = F.relu(ref)
    wp, _, _ = ops.pack_weight(wt)
    wp = wp.cuda()
    xd = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    cfgs = [c for c in tuning.RRG_CFGS
            if N.lib().dml_conv_rrg_fits(C.byref(_args(xd, wp, wp, xd, cin, cin, cout, kh, kw, ph, pw)), c)]
    assert cfgs, "no generic row-ring config takes this class"
    for cfg in cfgs:
        y = ops.conv2d_nhwc(xd, wp, b.cuda(), cout, kh, kw, (1, 1), (ph, pw), relu=relu, cfg=cfg)
        torch.cuda.synchronize()
        got = y[..., :cout].float().cpu().permute(0, 3, 1, 2)
        assert _rel(got, ref) < 1.5e-2, (cfg, _rel(got, ref))


def test_rrg_channel_offsets():
    """Input from a channel slice of a wider buffer, output into a channel slice (concat)."""
    torch.manual_seed(2)
    n, h, w = 2, 17, 17
    xfull = _bf(torch.randn(n, 192, h, w))
    x = xfull[:, 32:32 + 128]
    wt = _bf(torch.randn(96, 128, 1, 7) * (2.0 / 896) ** 0.5)
    b = torch.randn(96) * 0.1
    ref = F.relu(F.conv2d(x, wt, b, padding=(0, 3)))
    wp, _, _ = ops.pack_weight(wt)
    xd = xfull.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    for cfg in (160, 162, 164):
        out = torch.full((n, h, w, 160), 7.0, device="cuda", dtype=torch.bfloat16)
        ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), 96, 1, 7, (1, 1), (0, 3), relu=True, out=out, out_coff=40,
                        in_coff=32, cin=128, cfg=cfg)
        torch.cuda.synchronize()
        assert _rel(out[..., 40:136].float().cpu().permute(0, 3, 1, 2), ref) < 1.5e-2, cfg
        assert torch.all(out[..., :40] == 7.0) and torch.all(out[..., 136:] == 7.0), cfg


@pytest.mark.parametrize("bad", ["stride2", "residual", "f32", "pad"])
def test_rrg_refusals(bad):
    x = torch.zeros(2, 8, 8, 64, device="cuda", dtype=torch.bfloat16)
    wp, _, _ = ops.pack_weight(torch.zeros(64, 64, 3, 3))
    kw = dict(relu=True, cfg=160)
    if bad == "residual":
        kw["residual"] = torch.zeros(2, 8, 8, 64, device="cuda", dtype=torch.bfloat16)
    if bad == "f32":
        kw["out_f32"] = True
    with pytest.raises(N.NativeError, match="dml_conv_rrg"):
        ops.conv2d_nhwc(x, wp.cuda(), torch.zeros(64).cuda(), 64, 3, 3, (2, 2) if bad == "stride2" else (1, 1),
                        (1, 0) if bad == "pad" else (1, 1), **kw)
