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


# ------------------------------------------------------ InceptionV3 stem --
TH = TW = 16
R1H, R1W = TH + 2, TW + 2
IR_I, PQ_I = 2 * (R1H - 1) + 3, R1W + 1


def emulate_inception_stem(x_nhwc, k1_hwio, b1, k2_hwio, b2):
    """Tile math of inc_stem_kernel: 16x16 conv2 tiles, 18x18 conv1 window,
    37x19 pair-packed patch, conv1 K chunk c -> (row c >> 1 clamped to 2, pair
    tap c & 1) with zero weights on chunks 6, 7, conv2 k-step = tap (r, s)."""
    n_, h, w, _ = x_nhwc.shape
    w1 = pack_conv_weight(pair_pack_kernel(k1_hwio), 8, 32, 64)  # [32][64]: K = (r, s', c8) + 16 zero
    w2 = pack_conv_weight(k2_hwio, 32, 32, 320)[:, :288]          # [32][288]: K = (r, s, c)
    h1, wd1 = (h - 3) // 2 + 1, (w - 3) // 2 + 1
    h2, wd2 = h1 - 2, wd1 - 2
    y = np.zeros((n_, h2, wd2, 32), np.float32)
    p = np.arange(R1H * R1W)
    wa, wb = p // R1W, p % R1W
    for n in range(n_):
        for ty in range((h2 + TH - 1) // TH):
            for tx in range((wd2 + TW - 1) // TW):
                oy0, ox0 = ty * TH, tx * TW
                ir0, ic0 = 2 * oy0, 2 * ox0
                patch = np.zeros((IR_I, PQ_I, 8), np.float32)
                for i in range(IR_I):
                    ih = ir0 + i
                    if not 0 <= ih < h:
                        continue
                    for q in range(PQ_I):
                        iw = ic0 + 2 * q
                        if 0 <= iw < w:
                            patch[i, q, 0:3] = x_nhwc[n, ih, iw]
                        if 0 <= iw + 1 < w:
                            patch[i, q, 4:7] = x_nhwc[n, ih, iw + 1]
                chunks = []
                for c in range(8):
                    r, sp = min(c >> 1, 2), c & 1
                    chunks.append(patch[2 * wa + r, wb + sp])
                a1 = np.stack(chunks, 1).reshape(-1, 64)
                c1 = np.maximum(a1 @ w1.T + b1, 0.0)
                ok = (oy0 + wa < h1) & (ox0 + wb < wd1)
                c1 = np.where(ok[:, None], c1, 0.0).reshape(R1H, R1W, 32)
                taps = [c1[r:r + TH, s:s + TW] for r in range(3) for s in range(3)]
                a2 = np.stack(taps, 2).reshape(TH * TW, 288)
                out = np.maximum(a2 @ w2.T + b2, 0.0).reshape(TH, TW, 32)
                hh, ww = min(TH, h2 - oy0), min(TW, wd2 - ox0)
                y[n, oy0:oy0 + hh, ox0:ox0 + ww] = out[:hh, :ww]
    return y


@pytest.mark.parametrize("shape", [(1, 39, 41), (2, 35, 67)])
def test_inception_stem_tiling_matches_two_convs(shape):
    n, h, w = shape
    rng = np.random.default_rng(1)
    x = rng.standard_normal((n, h, w, 3)).astype(np.float32)
    k1 = (rng.standard_normal((3, 3, 3, 32)) * 0.3).astype(np.float32)
    b1 = (rng.standard_normal(32) * 0.1).astype(np.float32)
    k2 = (rng.standard_normal((3, 3, 32, 32)) * 0.1).astype(np.float32)
    b2 = (rng.standard_normal(32) * 0.1).astype(np.float32)
    t = F.relu(F.conv2d(torch.from_numpy(x).permute(0, 3, 1, 2), torch.from_numpy(k1).permute(3, 2, 0, 1),
                        torch.from_numpy(b1), stride=2))
    ref = F.relu(F.conv2d(t, torch.from_numpy(k2).permute(3, 2, 0, 1), torch.from_numpy(b2)))
    ref = ref.permute(0, 2, 3, 1).numpy()
    got = emulate_inception_stem(x, k1, b1, k2, b2)
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)
