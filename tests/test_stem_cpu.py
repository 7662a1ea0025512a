"""CPU model of the fused ResNet stem's tiling (csrc/kernels/stem_fused.hip):
7x8 pool-output blocks, the 15x17 conv window under them, the 35x20 pair-packed
input patch, fragment addressing patch[2a + r][b + s'] against the pair-packed
weight layout K = (r, s', c8), zeroed out-of-image conv positions and the 3x3/2
max pool from the window. The numpy emulation must reproduce
conv2d(7x7/2, pad 3) + bias + ReLU + max_pool2d(3, 2, pad 1) exactly (fp32),
including partial blocks at the image edges."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from distributed_machine_learning_amd.models.engine import pack_conv_weight, pair_pack_kernel

PH, PW = 7, 8
CR, CC = 2 * PH + 1, 2 * PW + 1
IR, PQ = 2 * (CR - 1) + 7, CC + 3


def emulate_stem(x_nhwc: np.ndarray, kernel_hwio: np.ndarray, bias: np.ndarray) -> np.ndarray:
    n_, h, w, _ = x_nhwc.shape
    wpk = pack_conv_weight(pair_pack_kernel(kernel_hwio), 8, 64, 224)  # [64][224], K = (r, s', c8)
    hc, wc = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    ho, wo = (hc - 1) // 2 + 1, (wc - 1) // 2 + 1
    y = np.zeros((n_, ho, wo, 64), np.float32)
    p = np.arange(CR * CC)
    wa, wb = p // CC, p % CC
    for n in range(n_):
        for by in range((ho + PH - 1) // PH):
            for bx in range((wo + PW - 1) // PW):
                py0, px0 = by * PH, bx * PW
                cr0, cc0 = 2 * py0 - 1, 2 * px0 - 1
                ir0, ic0 = 2 * cr0 - 3, 2 * cc0 - 3
                patch = np.zeros((IR, PQ, 8), np.float32)
                for i in range(IR):
                    ih = ir0 + i
                    if not 0 <= ih < h:
                        continue
                    for q in range(PQ):
                        iw = ic0 + 2 * q
                        if 0 <= iw < w:
                            patch[i, q, 0:3] = x_nhwc[n, ih, iw]
                        if 0 <= iw + 1 < w:
                            patch[i, q, 4:7] = x_nhwc[n, ih, iw + 1]
                # fragment gather: k-step r = kernel row, lane quarter = pair tap s'
                a = np.stack([np.stack([patch[2 * wa + r, wb + s] for s in range(4)], 1) for r in range(7)], 1)
                conv = np.maximum(a.reshape(CR * CC, 224) @ wpk.T + bias, 0.0)
                ok = (cr0 + wa >= 0) & (cr0 + wa < hc) & (cc0 + wb >= 0) & (cc0 + wb < wc)
                tile = np.where(ok[:, None], conv, 0.0).reshape(CR, CC, 64)
                for ly in range(PH):
                    for lx in range(PW):
                        oy, ox = py0 + ly, px0 + lx
                        if oy < ho and ox < wo:
                            y[n, oy, ox] = tile[2 * ly:2 * ly + 3, 2 * lx:2 * lx + 3].max((0, 1))
    return y


@pytest.mark.parametrize("shape", [(2, 32, 40), (1, 29, 31), (1, 61, 17)])
def test_stem_tiling_matches_conv_pool(shape):
    n, h, w = shape
    rng = np.random.default_rng(0)
    x = rng.standard_normal((n, h, w, 3)).astype(np.float32)
    k = (rng.standard_normal((7, 7, 3, 64)) * 0.2).astype(np.float32)
    b = (rng.standard_normal(64) * 0.1).astype(np.float32)
    ref = F.conv2d(torch.from_numpy(x).permute(0, 3, 1, 2), torch.from_numpy(k).permute(3, 2, 0, 1),
                   torch.from_numpy(b), stride=2, padding=3)
    ref = F.max_pool2d(F.relu(ref), 3, 2, 1).permute(0, 2, 3, 1).numpy()
    got = emulate_stem(x, k, b)
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)
