"""CPU model of the patch-stationary conv kernel's index math (csrc/kernels/conv_igemm_pt.hip):
M tiles of whole output rows / whole images, one zero-padded input patch per image and
channel chunk, each tap read at row offset r * PW + s. The model runs the kernel's geometry
(pt_geometry), its loader mapping (patch row -> input pixel or zero) and its MFMA-side
mapping (output pixel + tap -> patch row) in numpy and must reproduce a direct convolution
for every shape class the tuner offers it (3x3 / 5x5 / 1x7 / 7x1 / 1x3 / 3x1, 'same' and
'valid', multi-image tiles with a partial last tile, row blocks with a partial last block)."""
import numpy as np
import pytest


def geometry(N, Ho, Wo, kh, kw, BM):
    """pt_geometry: (TI, TH, PH, PW, PR, tiles per image, M tiles)."""
    if Ho * Wo <= BM:
        TI, TH, tpi = BM // (Ho * Wo), Ho, 1
        mt = -(-N // TI)
    else:
        TI, TH = 1, BM // Wo
        tpi = -(-Ho // TH)
        mt = N * tpi
    PH, PW = TH + kh - 1, Wo + kw - 1
    return TI, TH, PH, PW, TI * PH * PW, tpi, mt


def model_conv(x, w, ph, pw, BM, BK, prmax):
    """x [N,H,W,C], w [Co,kh,kw,C] -> y [N,Ho,Wo,Co] through the kernel's tiles."""
    N, H, W, C = x.shape
    Co, kh, kw, _ = w.shape
    Ho, Wo = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    TI, TH, PH, PW, PR, tpi, mt = geometry(N, Ho, Wo, kh, kw, BM)
    assert PR <= prmax and C % BK == 0
    y = np.zeros((N * Ho * Wo, Co), np.int64)
    for tm in range(mt):
        if TI > 1 or tpi == 1:
            n0, oh0, cnt = tm * TI, 0, min(TI, N - tm * TI) * Ho * Wo
        else:
            n0, oh0 = tm // tpi, (tm % tpi) * TH
            cnt = min(TH, Ho - oh0) * Wo
        m0 = n0 * Ho * Wo + oh0 * Wo
        for cb in range(C // BK):
            patch = np.zeros((prmax, BK), np.int64)     # loader: patch rows (dummy rows stay zero)
            for row in range(PR):
                ti, rem = divmod(row, PH * PW)
                prow, pcol = divmod(rem, PW)
                n, ih, iw = n0 + ti, oh0 - ph + prow, pcol - pw
                if n < N and 0 <= ih < H and 0 <= iw < W:
                    patch[row] = x[n, ih, iw, cb * BK:(cb + 1) * BK]
            for t in range(kh * kw):                    # MFMA waves: one K tile per tap
                tr, tcol = divmod(t, kw)
                toff = tr * PW + tcol
                for r in range(cnt):
                    ti, rem = divmod(r, TH * Wo)
                    ohl, ow = divmod(rem, Wo)
                    pb = (ti * PH + ohl) * PW + ow
                    y[m0 + r] += w[:, tr, tcol, cb * BK:(cb + 1) * BK] @ patch[pb + toff]
    return y.reshape(N, Ho, Wo, Co)


def direct_conv(x, w, ph, pw):
    N, H, W, C = x.shape
    Co, kh, kw, _ = w.shape
    xp = np.zeros((N, H + 2 * ph, W + 2 * pw, C), np.int64)
    xp[:, ph:ph + H, pw:pw + W] = x
    Ho, Wo = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    y = np.zeros((N, Ho, Wo, Co), np.int64)
    for r in range(kh):
        for s in range(kw):
            y += np.einsum("nhwc,oc->nhwo", xp[:, r:r + Ho, s:s + Wo], w[:, r, s])
    return y


@pytest.mark.parametrize("case", [
    # N, H, W, C, Co, kh, kw, ph, pw, BM, prmax
    (3, 14, 14, 128, 8, 3, 3, 1, 1, 256, 416),   # 196 px per image: one image per tile
    (11, 7, 7, 64, 8, 3, 3, 1, 1, 256, 416),     # 5 images per tile, partial last tile
    (2, 23, 19, 64, 8, 3, 3, 1, 1, 128, 240),    # row blocks (6 rows of 19), partial last block
    (2, 9, 9, 64, 8, 1, 7, 0, 3, 256, 416),      # 1x7 'same'
    (2, 9, 9, 64, 8, 7, 1, 3, 0, 256, 416),      # 7x1 'same'
    (3, 8, 8, 64, 8, 1, 3, 0, 1, 256, 416),      # 1x3 on 8x8: 4 images per tile
    (2, 12, 12, 64, 8, 5, 5, 2, 2, 128, 240),    # 5x5 'same'
    (2, 13, 11, 64, 8, 3, 3, 0, 0, 128, 240),    # 'valid'
])
def test_patch_model_matches_direct_conv(case):
    N, H, W, C, Co, kh, kw, ph, pw, BM, prmax = case
    rng = np.random.default_rng(0)
    x = rng.integers(-3, 4, size=(N, H, W, C))
    w = rng.integers(-3, 4, size=(Co, kh, kw, C))
    assert np.array_equal(model_conv(x, w, ph, pw, BM, 64, prmax), direct_conv(x, w, ph, pw))


def test_patch_sizes_of_the_served_layers():
    """The patch of every stride-1 layer the 256-pixel configs take fits their 416 rows."""
    layers = [(56, 56, 3, 3), (28, 28, 3, 3), (14, 14, 3, 3), (7, 7, 3, 3),       # ResNet50
              (35, 35, 3, 3), (17, 17, 1, 7), (17, 17, 7, 1), (8, 8, 1, 3), (8, 8, 3, 1), (8, 8, 3, 3),
              (71, 71, 3, 3)]                                                     # InceptionV3
    for Ho, Wo, kh, kw in layers:
        assert geometry(128, Ho, Wo, kh, kw, 256)[4] <= 416, (Ho, Wo, kh, kw)
    assert geometry(128, 35, 35, 5, 5, 256)[4] > 416          # the 5x5 branch: refused, v2 / ws take it
