"""CPU model of the generic row-ring conv kernel's index math (csrc/kernels/conv_rowring.hip,
namespace rrg, cfg 160..177): the launcher's geometry (dml_conv_rrg_geometry, host code), the
loader waves' DMA into the swizzled weight block and the channel-group planes of the row ring,
the MFMA waves' fragment addresses and the accumulator epilogue, replayed in numpy against a
plain fp32 convolution. The replay lands tile t+1's rows in LDS BEFORE tile t reads (the DMA is
issued right after tile t's barrier), so a ring slot that tile t still needs would be caught.
Also: the chunk swizzle is conflict-free for 16 consecutive 64-B rows at any start (the
ds_read_b128 lane groups of the MI355X LDS table)."""
import ctypes as C

import numpy as np
import pytest

from distributed_machine_learning_amd import _native as N

SHAPES = {i: s for i, s in enumerate([(2, 2, 2, 7, 2), (1, 4, 2, 3, 2), (1, 4, 3, 2, 2), (1, 4, 4, 2, 2),
                                       (2, 2, 1, 5, 2), (1, 4, 2, 4, 2), (2, 4, 2, 2, 2), (1, 8, 2, 2, 2),
                                       (1, 4, 3, 3, 2)])}  # WC, WP, FI, FJ, NL (DML_RRG_CFGS)


def key(row):
    return (row >> 1) & 2


def xcd_remap(b, nb):
    xcd, q, r = b & 7, nb >> 3, nb & 7
    base = xcd * (q + 1) if xcd < r else r * (q + 1) + (xcd - r) * q
    return base + (b >> 3)


def args(n, h, w, cin, ldx, cout, kh, kw, ph, pw, kpad):
    ho, wo = h + 2 * ph - kh + 1, w + 2 * pw - kw + 1
    return N.ConvArgs(None, None, None, None, None, n, h, w, cin, ldx, kh, kw, 1, 1, ph, pw, ho, wo, cout,
                      kh * kw * cin, kpad, cout, 0, 1, 0, 1, 1)


def geometry(a, cfg):
    out = (C.c_int * 12)()
    if N.lib().dml_conv_rrg_geometry(C.byref(a), cfg, out) != 0:
        return None
    return dict(zip("CG SLOTP RING TH strips ncc wbytes plane ntile taps lds grid".split(), list(out)))


def replay(a, cfg, g, x, wp, bias):
    """The kernel, workgroup by workgroup, on a float LDS image (2-byte cells)."""
    WC, WP, FI, FJ, NL = SHAPES[(cfg - 160) // 2]
    cout_wg = WC * FI * 16
    y = np.full((a.N, a.Ho, a.Wo, a.Cout), np.nan, np.float32)
    lane = np.arange(64)
    lrow, lq = lane >> 2, lane & 3
    lchunk = lq ^ key(lrow)
    frow, fq = lane & 15, lane >> 4
    xf = x.reshape(-1)
    for b in range(g["grid"]):
        lds = np.full(g["lds"] // 2, np.nan, np.float32)   # never-written cells poison the result
        L = xcd_remap(b, g["grid"])
        cc, sidx = L % g["ncc"], L // g["ncc"]
        n, sp = sidx // g["strips"], sidx % g["strips"]
        t0, t1 = sp * g["ntile"] // g["strips"], (sp + 1) * g["ntile"] // g["strips"]
        TH, RING, SLOTP, CG = g["TH"], g["RING"], g["SLOTP"], g["CG"]
        gbase = t0 * TH - a.ph
        c0 = cc * cout_wg

        def dma(dst_byte, vals):          # one 1-KiB piece: lane L writes 16 B at dst + 16 L
            idx = dst_byte // 2 + (lane[:, None] * 8 + np.arange(8)[None, :])
            lds[idx] = vals

        for p in range(g["taps"] * CG * cout_wg // 16):
            row = p * 16 + lrow
            tg, cl = row // cout_wg, row % cout_wg
            tap, gg = tg // CG, tg % CG
            ch, co = gg * 32 + lchunk * 8, c0 + cl
            ok = (ch < a.Cin) & (co < a.Cout)
            k = tap * a.Cin + ch
            v = np.where(ok[:, None], wp[np.minimum(co, wp.shape[0] - 1)[:, None],
                                         np.minimum(k[:, None] + np.arange(8), wp.shape[1] - 1)], 0.0)
            dma(p * 1024, v)
        ppr = SLOTP // 16

        def rows(r0, cnt):
            for p in range(cnt * CG * ppr):
                rr, rem = p // (CG * ppr), p % (CG * ppr)
                gg, pc = rem // ppr, rem % ppr
                gr = r0 + rr
                slot = (gr - gbase) % RING
                col = pc * 16 + lrow
                iw, ch = col - a.pw, gg * 32 + lchunk * 8
                ok = (0 <= gr < a.H) & (iw >= 0) & (iw < a.W) & (ch < a.Cin)
                off = (((n * a.H + gr) * a.W + iw) * a.ldx + ch)
                v = np.where(ok[:, None], xf[np.where(ok, off, 0)[:, None] + np.arange(8)], 0.0)
                dma(g["wbytes"] + gg * g["plane"] + (slot * SLOTP + pc * 16) * 64, v)

        if t0 < t1:
            rows(gbase, TH + a.kh - 1)
        tpx = TH * a.Wo
        nfrag = (tpx + 15) // 16
        for t in range(t0, t1):
            if t + 1 < t1:   # tile t+1's rows land before tile t reads
                rows((t + 1) * TH - a.ph + a.kh - 1, TH)
            r0 = t * TH
            cnt = min(TH, a.Ho - r0) * a.Wo
            s0 = ((t - t0) * TH) % RING
            for wid in range(WC * WP):
                wc, wpp = wid % WC, wid // WC
                cw = c0 + wc * FI * 16
                aoff = (wc * FI * 16 + frow) * 64 + ((fq ^ key(frow)) << 4)
                for j in range(FJ):
                    fj = j * WP + wpp
                    if fj >= nfrag:
                        continue
                    p = fj * 16 + frow
                    p = np.where(p < tpx, p, 0)
                    ohl, ow = p // a.Wo, p % a.Wo
                    sl = s0 + ohl
                    sl = np.where(sl >= RING, sl - RING, sl)
                    acc = np.zeros((FI, 16, 16), np.float64)
                    for st in range(g["taps"] * CG):
                        tap, gg = st // CG, st % CG
                        r, sx = tap // a.kw, tap % a.kw
                        v = sl + r
                        v = np.where(v >= RING, v - RING, v)
                        P = v * SLOTP + ow + sx
                        boff = g["wbytes"] + gg * g["plane"] + P * 64 + ((fq ^ key(P)) << 4)
                        B = lds[boff[:, None] // 2 + np.arange(8)]          # lane -> 8 k values
                        Bm = np.zeros((32, 16))
                        Bm[fq[:, None] * 8 + np.arange(8), frow[:, None]] = B
                        for i in range(FI):
                            A = lds[(st * cout_wg * 64 + aoff + i * 16 * 64)[:, None] // 2 + np.arange(8)]
                            Am = np.zeros((16, 32))
                            Am[frow[:, None], fq[:, None] * 8 + np.arange(8)] = A
                            acc[i] += Am @ Bm
                    for i in range(FI):
                        for ln in range(64):
                            lp = fj * 16 + (ln & 15)
                            if lp >= cnt:
                                continue
                            m = r0 * a.Wo + lp
                            oh, ow_ = m // a.Wo, m % a.Wo
                            for e in range(4):
                                c = cw + i * 16 + (ln >> 4) * 4 + e
                                if c < a.Cout:
                                    y[n, oh, ow_, c] = acc[i, (ln >> 4) * 4 + e, ln & 15] + bias[c]
    return y


CASES = [  # n, h, w, cin, cout, kh, kw, same
    (1, 9, 9, 64, 64, 3, 3, True),
    (2, 7, 11, 80, 48, 3, 3, False),     # conv2d_5's class: Cin 80 (a half plane), valid
    (1, 9, 9, 48, 64, 5, 5, True),       # 5x5 Cin 48
    (1, 6, 17, 40, 32, 1, 7, True),
    (1, 17, 6, 40, 32, 7, 1, True),
    (1, 8, 8, 96, 96, 3, 3, True),
    (2, 5, 30, 32, 16, 3, 1, True),      # wide row, Cout below a chunk
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("inst", [0, 1, 2, 8])
def test_rrg_model_matches_conv(case, inst):
    n, h, w, cin, cout, kh, kw, same = case
    rng = np.random.default_rng(0)
    ph, pw = ((kh - 1) // 2, (kw - 1) // 2) if same else (0, 0)
    ldx = cin + 8          # input channel slice of a wider buffer
    x = np.zeros((n, h, w, ldx), np.float32)
    x[..., :cin] = rng.standard_normal((n, h, w, cin))
    x[..., cin:] = np.nan  # never read
    wt = rng.standard_normal((cout, cin, kh, kw)).astype(np.float32)
    kpad = (kh * kw * cin + 63) // 64 * 64
    wp = np.zeros(((cout + 255) // 256 * 256, kpad), np.float32)
    wp[:cout, :kh * kw * cin] = wt.transpose(0, 2, 3, 1).reshape(cout, -1)
    bias = rng.standard_normal(cout).astype(np.float32)
    a = args(n, h, w, cin, ldx, cout, kh, kw, ph, pw, kpad)
    for cfg in (160 + 2 * inst, 161 + 2 * inst):
        g = geometry(a, cfg)
        if g is None:
            continue
        got = replay(a, cfg, g, x, wp, bias)
        xp = np.pad(x[..., :cin], ((0, 0), (ph, ph), (pw, pw), (0, 0)))
        ref = np.zeros_like(got)
        for r in range(kh):
            for s in range(kw):
                ref += np.einsum("nhwc,oc->nhwo", xp[:, r:r + a.Ho, s:s + a.Wo], wt[:, :, r, s])
        ref += bias
        assert np.isfinite(got).all(), (cfg, g)
        assert np.allclose(got, ref, atol=1e-3, rtol=1e-4), (cfg, g, np.abs(got - ref).max())


def test_rrg_geometry_and_refusals():
    # conv2d_5 (b64): 80 -> 192, 3x3 valid, 73 -> 71: a 32-cout chunk fits 2 rows per tile
    g = geometry(args(64, 73, 73, 80, 80, 192, 3, 3, 0, 0, 768), 162)
    assert g is not None and g["CG"] == 3 and g["SLOTP"] == 80 and g["ncc"] == 6 and g["lds"] <= 163840
    assert g["TH"] >= 1 and g["RING"] == 2 * g["TH"] + 2
    assert geometry(args(2, 8, 8, 64, 64, 64, 3, 3, 1, 1, 576), 160) is not None
    bad = args(2, 8, 8, 64, 64, 64, 3, 3, 1, 1, 576)
    bad.sh = bad.sw = 2
    assert geometry(bad, 160) is None                                  # stride 2
    assert geometry(args(2, 8, 8, 64, 64, 64, 3, 3, 1, 0, 576), 160) is None   # neither same nor valid
    big = args(2, 8, 8, 512, 512, 512, 3, 3, 1, 1, 4608)
    assert geometry(big, 160) is None                                  # weight block > 160 KiB
    assert N.lib().dml_conv_rrg_bn(164) == 48 and N.lib().dml_conv_rrg_bn(159) == 0


def test_swizzle_conflict_free_any_start():
    groups = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
              list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
    groups += [[lane + 32 for lane in gr] for gr in groups]
    for p0 in range(64):
        for gr in groups:
            quads = {((p0 + (ln & 15)) * 4 + ((ln >> 4) ^ key(p0 + (ln & 15)))) % 16 for ln in gr}
            assert len(quads) == 16, p0
