"""Whole-bottleneck fused kernel (csrc/kernels/block_fused.hip) against (a) the
same block run as three native conv launches (reduce, 3x3, expand + shortcut)
and (b) a plain-PyTorch fp32 reference with the intermediates rounded to bf16
where the unfused path stores them. Shapes: ResNet50 stage 2 (56x56, C 256),
tiles that straddle the image edge (20x20, 30x23) and stage 3's 28x28 grid."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from distributed_machine_learning_amd import ops  # noqa: E402


def _bf(x):
    return x.to(torch.bfloat16).float()


def _block_params(f, seed):
    g = torch.Generator().manual_seed(seed)
    c = 4 * f
    w1 = torch.randn(f, c, 1, 1, generator=g) * (2.0 / c) ** 0.5
    w2 = torch.randn(f, f, 3, 3, generator=g) * (2.0 / (9 * f)) ** 0.5
    w3 = torch.randn(c, f, 1, 1, generator=g) * (0.5 / f) ** 0.5
    b1, b2, b3 = (torch.randn(k, generator=g) * 0.1 for k in (f, f, c))
    return w1, w2, w3, b1, b2, b3


def _reference(x, w1, w2, w3, b1, b2, b3):
    """fp32 NCHW reference; T1/T2 rounded to bf16 (the unfused kernels store them so)."""
    xc = x.float().permute(0, 3, 1, 2)
    t1 = _bf(F.relu(F.conv2d(xc, _bf(w1), b1)))
    t2 = _bf(F.relu(F.conv2d(t1, _bf(w2), b2, padding=1)))
    y = F.relu(F.conv2d(t2, _bf(w3), b3) + xc)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("kernel", [0, 1])
@pytest.mark.parametrize("n,h,w", [(2, 56, 56), (1, 20, 20), (3, 30, 23), (1, 28, 28), (5, 56, 56)])
def test_block_fused_matches_unfused_and_fp32(n, h, w, kernel):
    f = 64
    c = 4 * f
    dev = "cuda"
    w1, w2, w3, b1, b2, b3 = _block_params(f, seed=n * 100 + h)
    x = torch.randn(n, h, w, c, generator=torch.Generator().manual_seed(7)).to(torch.bfloat16).to(dev)
    w1p, w2p, w3p = (ops.pack_weight(t)[0].to(dev) for t in (w1, w2, w3))
    y = ops.block_fused(x, w1p, b1, w2p, b2, w3p, b3, kernel=kernel)
    # the three-launch path of the same block
    t1 = ops.conv2d_nhwc(x, w1p, b1, f, 1, 1, relu=True)
    t2 = ops.conv2d_nhwc(t1, w2p, b2, f, 3, 3, pad=(1, 1), relu=True)
    y3 = ops.conv2d_nhwc(t2, w3p, b3, c, 1, 1, relu=True, residual=x)
    torch.cuda.synchronize()
    ref = _reference(x.cpu(), w1, w2, w3, b1, b2, b3)
    got = y.float().cpu()
    d3 = (got - y3.float().cpu()).abs().max().item()
    rel = ((got - ref).abs().max() / ref.abs().max()).item()
    # same K order and bf16 intermediates as the unfused kernels: within one bf16 ulp
    assert d3 <= 2 ** -7 * y3.float().abs().max().item(), d3
    assert rel < 1e-2, rel


def test_block_fused_rejects_unsupported():
    from distributed_machine_learning_amd._native import NativeError

    x = torch.zeros(1, 14, 14, 512, dtype=torch.bfloat16, device="cuda")  # F = 128: not instantiated
    w = torch.zeros(512, 1152, dtype=torch.bfloat16, device="cuda")
    b = torch.zeros(512)
    with pytest.raises(NativeError):
        ops.block_fused(x, w, b, w, b, w, b)
