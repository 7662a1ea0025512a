"""Winograd F(2x2, 3x3) on the CPU: the host filter transform + fragment packing
(ops/winograd.py) against what csrc/kernels/conv_wino.hip reads, and the
kernel's arithmetic model (fp32 transforms, bf16-rounded V and U, fp32 GEMMs)
against a plain fp32 conv — the error budget the GPU kernel is held to."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from distributed_machine_learning_amd.ops import winograd as W

CASES = [  # n, h, w, cin, cout, pad
    (2, 9, 11, 64, 96, 1), (1, 7, 7, 40, 64, 1), (2, 10, 9, 80, 72, 0), (1, 14, 14, 256, 256, 1),
    (1, 8, 8, 448, 384, 1), (1, 73, 73, 80, 192, 0),
]


def _ref(x, k, b, pad):
    return F.conv2d(torch.from_numpy(x).permute(0, 3, 1, 2), torch.from_numpy(k).permute(3, 2, 0, 1),
                    torch.from_numpy(b), padding=pad).permute(0, 2, 3, 1).numpy()


def _rel(a, b):
    return float(np.abs(a - b).max() / np.abs(b).max())


@pytest.mark.parametrize("case", CASES)
def test_transform_exact_and_bf16_error_budget(case):
    n, h, w, ci, co, pad = case
    rng = np.random.default_rng(hash(case) % 2**32)
    x = W._bf16(rng.standard_normal((n, h, w, ci)).astype(np.float32))
    k = W._bf16(rng.standard_normal((3, 3, ci, co)).astype(np.float32) * (2 / (9 * ci)) ** 0.5)
    b = rng.standard_normal(co).astype(np.float32) * 0.1
    ref = _ref(x, k, b, pad)
    u = W.filter_transform(k)
    assert _rel(W.conv_model(x, u, b, pad, False, round_v=False), ref) < 1e-5   # the algebra is exact
    model = W.conv_model(x, W._bf16(u), b, pad, True)
    assert _rel(model, np.maximum(ref, 0)) < 1e-2                               # bf16 V and U: well inside 1.5e-2


@pytest.mark.parametrize("ci,co", [(64, 64), (80, 192), (448, 384), (40, 8)])
@pytest.mark.parametrize("tn", [32, 64])
def test_packing_matches_kernel_addressing(ci, co, tn):
    rng = np.random.default_rng(ci * 1000 + co)
    u = rng.standard_normal((16, ci, co)).astype(np.float32)
    p = W.pack(u)
    assert p.shape == (-(-ci // 32), 16, -(-co // 64) * 4, 64, 8)
    assert np.array_equal(W.unpack(p, ci, co, tn), u)
    # padding rows/cols are zero (the kernel multiplies the channel tail / extra fragments by them)
    full = W.unpack(p, p.shape[0] * 32, p.shape[2] * 16, tn)
    assert not full[:, ci:].any() and not full[:, :, co:].any()


def test_ops_pack_wino_weight_matches_numpy():
    from distributed_machine_learning_amd import ops

    torch.manual_seed(0)
    w = torch.randn(96, 64, 3, 3)
    got = ops.pack_wino_weight(w)
    want = W.pack_kernel(w.permute(2, 3, 1, 0).numpy())
    assert got.dtype == torch.bfloat16 and got.numel() == want.size
    assert torch.equal(got, torch.from_numpy(want.reshape(-1)).to(torch.bfloat16))
