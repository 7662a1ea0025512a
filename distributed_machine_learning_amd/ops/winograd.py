"""Winograd F(2x2, 3x3) on the host: filter transform, fragment packing, and a
CPU model of what csrc/kernels/conv_wino.hip computes.

For a 2x2 output tile with 4x4 input window d and 3x3 filter g (correlation,
as conv layers compute it):

    Y = A^T [ (G g G^T) ⊙ (B^T d B) ] A

with the Lavin-Gray matrices below. The kernel receives U = G g G^T already
transformed (fp32 here, rounded once to bf16) and packed in the order its waves
read MFMA A fragments: [Cin/32][16 positions][Cout/16 fragments][64 lanes][8],
lane l of fragment f holding output channel 16f + (l & 15) and input channels
8(l >> 4) .. +8 of the chunk (v_mfma_f32_16x16x32_bf16's A layout).
"""
from __future__ import annotations

import numpy as np

BT = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], np.float32)
G = np.array([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], np.float32)
AT = np.array([[1, 1, 1, 0], [0, 1, -1, -1]], np.float32)

KC = 32  # input channels per chunk (conv_wino.hip)


def filter_transform(k_hwio: np.ndarray) -> np.ndarray:
    """[3, 3, cin, cout] fp32 -> U [16, cin, cout] fp32, position p = 4a + b."""
    assert k_hwio.shape[:2] == (3, 3), k_hwio.shape
    u = np.einsum("ar,rsio,bs->abio", G, k_hwio.astype(np.float32), G)
    return u.reshape(16, *k_hwio.shape[2:])


def nfrag(cout: int) -> int:
    """16-channel fragments of the packed layout (Cout padded to a multiple of 64, so any
    configuration's 32- or 64-channel tile reads inside it)."""
    return -(-cout // 64) * 4


def pack(u: np.ndarray) -> np.ndarray:
    """U [16, cin, cout] -> the kernel's fragment order [nkc, 16, nfrag, 64, 8]: piece
    (chunk kc, position p, fragment f) is the 1-KiB A fragment of v_mfma_f32_16x16x32_bf16
    (lane l: output channel 16f + (l & 15), input channels 32kc + 8(l >> 4) .. +8); zero-padded."""
    _, cin, cout = u.shape
    nkc, nft = -(-cin // KC), nfrag(cout)
    up = np.zeros((16, nkc * KC, nft * 16), np.float32)
    up[:, :cin, :cout] = u
    # cin = kc*32 + q*8 + e ; cout = f*16 + c16 ; lane = q*16 + c16
    v = up.reshape(16, nkc, 4, 8, nft, 16)               # pos, kc, q, e, f, c16
    v = v.transpose(1, 0, 4, 2, 5, 3)                    # kc, pos, f, q, c16, e
    return np.ascontiguousarray(v.reshape(nkc, 16, nft, 64, 8))


def pack_kernel(k_hwio: np.ndarray) -> np.ndarray:
    return pack(filter_transform(k_hwio))


def unpack(packed: np.ndarray, cin: int, cout: int, tn: int = 32) -> np.ndarray:
    """Read the packed array back the way a workgroup of a ``tn``-channel configuration
    addresses it: output-channel tile ct, chunk kc, piece j = (position j // NF, fragment
    j % NF), lane l, element e."""
    nkc, _, nft = packed.shape[:3]
    nf = tn // 16
    u = np.zeros((16, nkc * KC, nft * 16), np.float32)
    lane = np.arange(64)
    flat = packed.reshape(-1, 64, 8)
    for ct in range(nft // nf):
        for kc in range(nkc):
            for j in range(16 * nf):
                p, f = j // nf, j % nf
                piece = (kc * 16 + p) * nft + ct * nf + f      # conv_wino.hip issue_w
                co = (ct * nf + f) * 16 + (lane & 15)
                for e in range(8):
                    u[p, kc * KC + (lane >> 4) * 8 + e, co] = flat[piece, :, e]
    return u[:, :cin, :cout]


def _bf16(x: np.ndarray) -> np.ndarray:
    import torch

    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(torch.bfloat16).float().numpy()


def conv_model(x_nhwc: np.ndarray, u: np.ndarray, bias: np.ndarray, pad: int, relu: bool,
               round_v: bool = True) -> np.ndarray:
    """The kernel's arithmetic on the CPU: input tiles transformed in fp32 and
    rounded once to bf16 (round_v), 16 fp32 GEMMs over the channels with the
    bf16 U, output transform + bias (+ ReLU) in fp32. x: [N, H, W, Cin]."""
    n, h, w, cin = x_nhwc.shape
    ho, wo = h + 2 * pad - 2, w + 2 * pad - 2
    th, tw = -(-ho // 2), -(-wo // 2)
    xp = np.zeros((n, 2 * th + 2, 2 * tw + 2, cin), np.float32)
    hh, ww = min(h, 2 * th + 2 - pad), min(w, 2 * tw + 2 - pad)
    xp[:, pad:pad + hh, pad:pad + ww] = x_nhwc[:, :hh, :ww]
    # d[n, ty, tx, r, c, cin]: the 4x4 window of every tile
    idx_r = (2 * np.arange(th))[:, None] + np.arange(4)[None]
    idx_c = (2 * np.arange(tw))[:, None] + np.arange(4)[None]
    d = xp[:, idx_r][:, :, :, idx_c]                      # n, th, 4, tw, 4, cin
    d = d.transpose(0, 1, 3, 2, 4, 5)                      # n, th, tw, 4, 4, cin
    v = np.einsum("ir,ntwrcz,jc->ntwijz", BT, d, BT).reshape(n, th, tw, 16, cin)
    if round_v:
        v = _bf16(v)
    m = np.einsum("ntwpz,pzo->ntwpo", v, u).reshape(n, th, tw, 4, 4, -1)
    y = np.einsum("ai,ntwijo,bj->ntwabo", AT, m, AT)       # n, th, tw, 2, 2, cout
    y = y.transpose(0, 1, 3, 2, 4, 5).reshape(n, 2 * th, 2 * tw, -1)[:, :ho, :wo]
    y = y + bias[None, None, None, :]
    return np.maximum(y, 0) if relu else y
