"""Row-ring 3x3 conv kernel of ResNet50 stage 2 (csrc/kernels/conv_rowring.hip, cfg 150..152):
numerics against a plain-PyTorch fp32 conv of the same bf16 inputs — batch 1 / odd batch,
image heights that leave a partial last 4-row tile and strips of unequal length, Cout < 64,
residual, no ReLU, fp32 output, channel-offset input / output — and the refusals (width != 56,
Cin != 64, Cout > 64, stride 2)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from distributed_machine_learning_amd import _native as N, ops  # noqa: E402
from distributed_machine_learning_amd.ops import tuning  # noqa: E402

from test_kernels_gpu import _bf, _rel  # noqa: E402

RR = list(tuning.RR_CFGS)
CASES = [
    # n, h, cout, relu, residual, out_f32
    (2, 56, 64, True, False, False),   # ResNet50 stage 2
    (3, 56, 64, True, True, False),    # residual
    (1, 30, 64, False, False, False),  # partial last tile (30 rows = 7 tiles + 2), no ReLU
    (2, 9, 48, True, False, False),    # 3 tiles: strips of 1 / 2 tiles, Cout 48
    (2, 56, 64, False, False, True),   # fp32 output
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("cfg", RR)
def test_rr_conv_matches_fp32(case, cfg):
    n, h, cout, relu, has_res, f32 = case
    torch.manual_seed(1)
    x = _bf(torch.randn(n, 64, h, 56))
    wt = _bf(torch.randn(cout, 64, 3, 3) * (2.0 / (64 * 9)) ** 0.5)
    b = torch.randn(cout) * 0.1
    ref = F.conv2d(x, wt, b, padding=1)
    res = _bf(torch.randn_like(ref)) if has_res else None
    if res is not None:
        ref = ref + res
    if relu:
        ref = F.relu(ref)
    wp, _, _ = ops.pack_weight(wt)
    xd = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    rd = res.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16) if res is not None else None
    y = ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), cout, 3, 3, (1, 1), (1, 1), relu=relu, residual=rd, cfg=cfg,
                        out_f32=f32)
    torch.cuda.synchronize()
    got = y[..., :cout].float().cpu().permute(0, 3, 1, 2)
    assert _rel(got, ref) < 1.5e-2, _rel(got, ref)


@pytest.mark.parametrize("cfg", RR)
def test_rr_channel_offsets(cfg):
    """Input from a channel slice of a wider buffer, output into a channel slice."""
    torch.manual_seed(2)
    n, h = 2, 12
    xfull = _bf(torch.randn(n, 128, h, 56))
    x = xfull[:, 64:]
    wt = _bf(torch.randn(64, 64, 3, 3) * (2.0 / 576) ** 0.5)
    b = torch.randn(64) * 0.1
    ref = F.relu(F.conv2d(x, wt, b, padding=1))
    wp, _, _ = ops.pack_weight(wt)
    xd = xfull.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16)
    out = torch.full((n, h, 56, 96), 7.0, device="cuda", dtype=torch.bfloat16)
    ops.conv2d_nhwc(xd, wp.cuda(), b.cuda(), 64, 3, 3, (1, 1), (1, 1), relu=True, out=out, out_coff=32, in_coff=64,
                    cin=64, cfg=cfg)
    torch.cuda.synchronize()
    assert _rel(out[..., 32:].float().cpu().permute(0, 3, 1, 2), ref) < 1.5e-2
    assert torch.all(out[..., :32] == 7.0)


def test_rr_matches_v2_tile():
    """Same inputs through the row-ring kernel and a v2 tile: same K order, so the outputs
    agree to bf16 rounding."""
    torch.manual_seed(4)
    x = torch.randn(4, 56, 56, 64, device="cuda").to(torch.bfloat16)
    wp, _, _ = ops.pack_weight(torch.randn(64, 64, 3, 3) * 0.06)
    b = torch.randn(64, device="cuda") * 0.1
    y0 = ops.conv2d_nhwc(x, wp.cuda(), b, 64, 3, 3, (1, 1), (1, 1), relu=True, cfg=15)
    y1 = ops.conv2d_nhwc(x, wp.cuda(), b, 64, 3, 3, (1, 1), (1, 1), relu=True, cfg=150)
    torch.cuda.synchronize()
    assert (y0.float() - y1.float()).abs().max().item() <= 0.02 * y0.float().abs().max().item()


@pytest.mark.parametrize("bad", ["w28", "cin128", "cout128", "stride2"])
def test_rr_refusals(bad):
    w = 28 if bad == "w28" else 56
    cin = 128 if bad == "cin128" else 64
    cout = 128 if bad == "cout128" else 64
    x = torch.zeros(2, 8, w, cin, device="cuda", dtype=torch.bfloat16)
    wp, _, _ = ops.pack_weight(torch.zeros(cout, cin, 3, 3))
    with pytest.raises(N.NativeError, match="dml_conv_rr"):
        ops.conv2d_nhwc(x, wp.cuda(), torch.zeros(cout).cuda(), cout, 3, 3, (2, 2) if bad == "stride2" else (1, 1),
                        (1, 1), cfg=150)
