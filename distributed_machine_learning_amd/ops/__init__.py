"""Functional wrappers over the hand-written gfx950 kernels (csrc/kernels/).

Each op takes/returns torch tensors on the HIP device and launches exactly one
native kernel on the current stream. There is NO PyTorch fallback: if the native
library is missing these raise (tests on the GPU box therefore prove the HIP
path ran). CPU-side fp32 oracles for each op live in ``ops.reference``.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

import torch

from .. import _native as N

__all__ = ["conv2d_nhwc", "conv_group", "pool3x3", "global_avgpool", "softmax_top5", "preprocess", "pack_weight",
           "resnet_stem", "inception_stem", "conv3x3_pool", "expand_reduce"]


def _r(x, m):
    return (x + m - 1) // m * m


def pack_weight(w_oihw: torch.Tensor, cin_eff: Optional[int] = None) -> Tuple[torch.Tensor, int, int]:
    """OIHW fp32 -> bf16 [Cout_pad][K_pad] in (r, s, c) order. Returns (w, K, Kpad)."""
    co, ci, kh, kw = w_oihw.shape
    cin_eff = cin_eff or _r(ci, 8)
    k = torch.zeros((co, kh, kw, cin_eff), dtype=torch.float32)
    k[..., :ci] = w_oihw.permute(0, 2, 3, 1).float().cpu()
    K = kh * kw * cin_eff
    out = torch.zeros((_r(co, 256), _r(K, 64)), dtype=torch.float32)
    out[:co, :K] = k.reshape(co, K)
    return out.to(torch.bfloat16), K, _r(K, 64)


def conv2d_nhwc(x: torch.Tensor, w_packed: torch.Tensor, bias: torch.Tensor, cout: int, kh: int, kw: int,
                stride=(1, 1), pad=(0, 0), relu: bool = False, residual: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None, out_coff: int = 0, in_coff: int = 0, cin: Optional[int] = None,
                out_f32: bool = False, cfg: int = -1, K: Optional[int] = None, dilation=(1, 1),
                out_hw: Optional[Tuple[int, int]] = None, ksplit: int = 1,
                defer: Optional[list] = None) -> torch.Tensor:
    """x: NHWC bf16 [N,H,W,Cbuf] (Cbuf % 8 == 0). Returns/updates NHWC output.
    defer: a list to append the ConvArgs to instead of launching (conv_group).
    ksplit > 1 (fp32 output, v2 cfg): returns the [ksplit, N, Ho, Wo, C] split-K
    partial sums (slice 0 carries the bias); their sum is the convolution."""
    n, h, w_, cbuf = x.shape
    cin = cin if cin is not None else cbuf - in_coff
    ho = (h + 2 * pad[0] - dilation[0] * (kh - 1) - 1) // stride[0] + 1
    wo = (w_ + 2 * pad[1] - dilation[1] * (kw - 1) - 1) // stride[1] + 1
    if out_hw is not None:
        ho, wo = out_hw
    parts = None
    if ksplit > 1:
        assert out_f32 and out is None, "split-K writes fp32 partial slices into its own buffer"
        parts = torch.empty((ksplit, n, ho, wo, _r(cout, 8)), device=x.device, dtype=torch.float32)
        out = parts[0]
    if out is None:
        out = torch.empty((n, ho, wo, _r(cout, 8)), device=x.device,
                          dtype=torch.float32 if out_f32 else torch.bfloat16)
    assert out.is_contiguous() and x.is_contiguous()
    kpad = w_packed.shape[1]
    K = K if K is not None else kh * kw * cin
    bias_p = torch.zeros(w_packed.shape[0], device=x.device, dtype=torch.float32)
    bias_p[: bias.numel()] = bias.to(x.device, torch.float32)
    esz = out.element_size()
    a = N.ConvArgs(x.data_ptr() + 2 * in_coff, w_packed.data_ptr(), bias_p.data_ptr(),
                   residual.data_ptr() if residual is not None else None, out.data_ptr() + esz * out_coff,
                   n, h, w_, cin, cbuf, kh, kw, stride[0], stride[1], pad[0], pad[1], ho, wo, cout, K, kpad,
                   out.shape[-1], residual.shape[-1] if residual is not None else 0, int(relu), int(out_f32),
                   dilation[0], dilation[1])
    if parts is not None:
        a.ksplit, a.split_ld = ksplit, out.numel()
    if residual is not None and residual.shape[1] != ho:  # shortcut read at stride rs (full-res grid)
        rs = residual.shape[1] // ho
        assert residual.shape[1] == ho * rs and residual.shape[2] == wo * rs and residual.is_contiguous()
        a.rsub, a.rW, a.rHW = rs, residual.shape[2], residual.shape[1] * residual.shape[2]
    L = N.lib()
    if defer is not None:
        defer.append(a)
        out._keep = bias_p
        return out
    if cfg < 0:
        cfg = L.dml_conv_pick_cfg(C.byref(a))
    N.check(L.dml_conv(C.byref(a), cfg, N.stream_ptr()), "dml_conv")
    if parts is not None:
        parts._keep = bias_p
        return parts
    out._keep = bias_p  # keep alive until the kernel ran (caller syncs)
    return out


def conv_group(args: list, cfg: int, pools: Optional[list] = None) -> None:
    """Launch up to GROUP_MAX independent convs (ConvArgs from conv2d_nhwc(...,
    defer=list)) and up to GROUP_POOL_MAX 3x3 pools (PoolArgs from pool3x3(...,
    defer=list)) as ONE grid on tile config ``cfg`` (dml_conv_group)."""
    from .tuning import group_args

    N.check(N.lib().dml_conv_group(C.byref(group_args(args, pools or [])), cfg, N.stream_ptr()), "dml_conv_group")


def pool3x3(x: torch.Tensor, mode: str, k: int = 3, stride: int = 2, pad: int = 0,
            out: Optional[torch.Tensor] = None, out_coff: int = 0, relu: bool = False,
            defer: Optional[list] = None) -> torch.Tensor:
    """defer: a list to append the PoolArgs to instead of launching (conv_group)."""
    n, h, w, c = x.shape
    ho = (h + 2 * pad - k) // stride + 1
    wo = (w + 2 * pad - k) // stride + 1
    if out is None:
        out = torch.empty((n, ho, wo, c), device=x.device, dtype=torch.bfloat16)
    a = N.PoolArgs(x.data_ptr(), out.data_ptr() + 2 * out_coff, n, h, w, c, c, ho, wo, out.shape[-1], k, stride, pad,
                   0 if mode == "max" else 1, int(relu))
    if defer is not None:
        defer.append(a)
        return out
    N.check(N.lib().dml_pool(C.byref(a), N.stream_ptr()), "dml_pool")
    return out


def global_avgpool(x: torch.Tensor) -> torch.Tensor:
    n, h, w, c = x.shape
    out = torch.empty((n, c), device=x.device, dtype=torch.bfloat16)
    N.check(N.lib().dml_global_avgpool(x.data_ptr(), out.data_ptr(), n, h * w, c, c, N.stream_ptr()), "gap")
    return out


def softmax_top5(logits: torch.Tensor, want_probs: bool = True):
    """logits [B, classes], or [S, B, classes] split-K partial slices (summed
    in the kernel; the sum is written back into slice 0)."""
    parts = logits.contiguous().float()
    if parts.dim() == 2:
        parts = parts[None]
    s, b, classes = parts.shape
    probs = torch.empty((b, classes), device=parts.device, dtype=torch.float32) if want_probs else None
    idx = torch.empty((b, 5), device=parts.device, dtype=torch.int32)
    p = torch.empty((b, 5), device=parts.device, dtype=torch.float32)
    N.check(N.lib().dml_softmax_top5_split(parts.data_ptr(), b, classes, classes, s, b * classes,
                                           probs.data_ptr() if probs is not None else None, idx.data_ptr(),
                                           p.data_ptr(), N.stream_ptr()), "softmax_top5")
    return probs, idx, p


def preprocess(images_u8: torch.Tensor, out_hw, mode: str, pair: bool = False, lpad: int = 0) -> torch.Tensor:
    """uint8 NHWC -> bf16 NHWC8. pair=True writes the pair-packed stem layout
    [n][h][lpad + w][pixel j-lpad (3ch), 0, pixel j-lpad+1 (3ch), 0]."""
    n, hs, ws, _ = images_u8.shape
    wout = out_hw[1] + (lpad if pair else 0)
    out = torch.empty((n, out_hw[0], wout, 8), device=images_u8.device, dtype=torch.bfloat16)
    a = N.PreprocArgs(images_u8.data_ptr(), out.data_ptr(), n, hs, ws, out_hw[0], out_hw[1],
                      0 if mode == "caffe" else 1, int(pair), lpad)
    N.check(N.lib().dml_preprocess(C.byref(a), N.stream_ptr()), "preprocess")
    return out


def resnet_stem(images_u8: torch.Tensor, w_packed: torch.Tensor, bias: torch.Tensor, out_hw=(224, 224),
                mode: str = "caffe", w4: Optional[torch.Tensor] = None, b4: Optional[torch.Tensor] = None):
    """Fused ResNet stem (csrc/kernels/stem_fused.hip): uint8 [N, Hs, Ws, 3] ->
    nearest resize to out_hw + caffe/tf normalisation -> conv 7x7/2 pad 3 with the
    pair-packed bf16 weights [>=64][>=224] (models.engine.pair_pack_kernel +
    pack_conv_weight) + bias + ReLU -> max pool 3x3/2 pad 1 -> bf16 NHWC [N, Ho, Wo, 64].
    With w4 (bf16 [>=64][>=64], packed) and b4: also the folded 1x1 conv relu(w4 . pool + b4)
    (ResNet50 conv2_block1_1); returns (pool, z) then."""
    n, hs, ws, _ = images_u8.shape
    h, w = out_hw
    hc, wc = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    ho, wo = (hc - 1) // 2 + 1, (wc - 1) // 2 + 1
    out = torch.empty((n, ho, wo, 64), device=images_u8.device, dtype=torch.bfloat16)
    bias_p = bias.to(images_u8.device, torch.float32).contiguous()
    assert images_u8.is_contiguous() and w_packed.is_contiguous() and w_packed.shape[0] >= 64
    a = N.StemArgs(images_u8.data_ptr(), w_packed.data_ptr(), bias_p.data_ptr(), out.data_ptr(), n, hs, ws, h, w,
                   0 if mode == "caffe" else 1, w_packed.shape[1], hc, wc, ho, wo, 64)
    z = None
    if w4 is not None:
        z = torch.empty((n, ho, wo, 64), device=images_u8.device, dtype=torch.bfloat16)
        b4p = b4.to(images_u8.device, torch.float32).contiguous()
        assert w4.is_contiguous() and w4.shape[0] >= 64
        a.w4, a.b4, a.z, a.c4, a.ldw4, a.ldz = w4.data_ptr(), b4p.data_ptr(), z.data_ptr(), 64, w4.shape[1], 64
    N.check(N.lib().dml_stem_resnet(C.byref(a), N.stream_ptr()), "dml_stem_resnet")
    out._keep = bias_p
    if z is not None:
        z._keep = b4p
        return out, z
    return out


def inception_stem(images_u8: torch.Tensor, w1_packed: torch.Tensor, b1: torch.Tensor, w2_packed: torch.Tensor,
                   b2: torch.Tensor, out_hw=(299, 299), mode: str = "tf") -> torch.Tensor:
    """Fused InceptionV3 stem (csrc/kernels/stem_fused.hip): uint8 [N, Hs, Ws, 3] ->
    nearest resize + normalisation -> conv 3x3/2 valid (pair-packed weights
    [>=32][>=64]) + ReLU -> conv 3x3 valid (weights [>=32][>=288], K = (r, s, 32 ch))
    + ReLU -> bf16 NHWC [N, H2, W2, 32]."""
    n, hs, ws, _ = images_u8.shape
    h, w = out_hw
    h1, w1 = (h - 3) // 2 + 1, (w - 3) // 2 + 1
    out = torch.empty((n, h1 - 2, w1 - 2, 32), device=images_u8.device, dtype=torch.bfloat16)
    b1p = b1.to(images_u8.device, torch.float32).contiguous()
    b2p = b2.to(images_u8.device, torch.float32).contiguous()
    assert images_u8.is_contiguous() and w1_packed.is_contiguous() and w2_packed.is_contiguous()
    a = N.IncStemArgs(images_u8.data_ptr(), w1_packed.data_ptr(), b1p.data_ptr(), w2_packed.data_ptr(),
                      b2p.data_ptr(), out.data_ptr(), n, hs, ws, h, w, 0 if mode == "caffe" else 1,
                      w1_packed.shape[1], w2_packed.shape[1], h1, w1, h1 - 2, w1 - 2, 32)
    N.check(N.lib().dml_stem_inception(C.byref(a), N.stream_ptr()), "dml_stem_inception")
    out._keep = (b1p, b2p)
    return out


def conv3x3_pool(x: torch.Tensor, w_packed: torch.Tensor, bias: torch.Tensor,
                 w4: Optional[torch.Tensor] = None, b4: Optional[torch.Tensor] = None,
                 c4: int = 0) -> torch.Tensor:
    """Fused conv 3x3 'same' (32 -> 64 channels, weights [>=64][>=288], K = (r, s, c))
    + bias + ReLU + max pool 3x3/2 'valid' (csrc/kernels/conv_pool.hip), optionally followed
    by a folded 1x1 conv 64 -> c4 (+ b4, ReLU; w4 packed [>=c4][>=64]).
    x: bf16 NHWC [N, H, W, Cbuf >= 32]; returns bf16 NHWC [N, Ho, Wo, 64 or c4]."""
    n, h, w, cbuf = x.shape
    ho, wo = (h - 3) // 2 + 1, (w - 3) // 2 + 1
    cy = c4 if c4 else 64
    out = torch.empty((n, ho, wo, cy), device=x.device, dtype=torch.bfloat16)
    bias_p = bias.to(x.device, torch.float32).contiguous()
    assert x.is_contiguous() and w_packed.is_contiguous()
    a = N.ConvPoolArgs(x.data_ptr(), w_packed.data_ptr(), bias_p.data_ptr(), out.data_ptr(), n, h, w, cbuf,
                       w_packed.shape[1], ho, wo, cy)
    keep = [bias_p]
    if c4:
        b4p = b4.to(x.device, torch.float32).contiguous()
        assert w4.is_contiguous() and w4.shape[0] >= c4
        a.w4, a.b4, a.c4, a.ldw4 = w4.data_ptr(), b4p.data_ptr(), c4, w4.shape[1]
        keep.append(b4p)
    N.check(N.lib().dml_conv3x3_pool(C.byref(a), N.stream_ptr()), "dml_conv3x3_pool")
    out._keep = keep
    return out


def expand_reduce(x: torch.Tensor, w3: torch.Tensor, b3: torch.Tensor, res: Optional[torch.Tensor],
                  w1: torch.Tensor, b1: torch.Tensor, c: Optional[int] = None, fz: int = 0):
    """Fused ResNet block boundary (csrc/kernels/expand_reduce_chain.hip), C = res channels,
    F = C / 4: y = relu(1x1 conv F -> C of x + b3 + res), z = relu(1x1 conv C -> F of y + b1).
    x: bf16 [..., F]; res: bf16 [..., C], C in {256, 512, 1024}; w3 [>=C][>=F], w1 [>=F][>=C]
    packed (pack_weight). Returns (y, z) with x's leading shape.
    res=None (merged projection shortcut): x is [..., 2F] (the [x ; s] concat), C = c = 256.
    fz: reduce width when it is not F — a stage's last boundary (C = 256, fz = 128: the next
    stage's first reduce; chained kernel)."""
    c = res.shape[-1] if res is not None else c
    f = fz or c // 4
    lead = x.shape[:-1]
    m = x.numel() // x.shape[-1]
    y = torch.empty((*lead, c), device=x.device, dtype=torch.bfloat16)
    z = torch.empty((*lead, f), device=x.device, dtype=torch.bfloat16)
    b3p = b3.to(x.device, torch.float32).contiguous()
    b1p = b1.to(x.device, torch.float32).contiguous()
    assert x.is_contiguous() and (res is None or res.is_contiguous()) and w3.is_contiguous() and w1.is_contiguous()
    assert w3.shape[0] >= c and w1.shape[0] >= f and b3p.numel() >= c and b1p.numel() >= f
    a = N.ExpandReduceArgs(x.data_ptr(), w3.data_ptr(), b3p.data_ptr(), res.data_ptr() if res is not None else None,
                           y.data_ptr(), w1.data_ptr(), b1p.data_ptr(), z.data_ptr(), m, x.shape[-1], w3.shape[1],
                           res.shape[-1] if res is not None else 0, c, w1.shape[1], f, c,
                           c // 4 if res is not None else c // 2)
    a.fz = f
    N.check(N.lib().dml_expand_reduce(C.byref(a), N.stream_ptr()), "dml_expand_reduce")
    y._keep = (b3p, b1p)
    return y, z


def fused_conv1x1(x: torch.Tensor, members, stride: int = 1, cfg: int = -1) -> None:
    """Sibling 1x1 convs on the same input as ONE segmented GEMM.
    members: list of (w_oihw fp32 [co, ci, 1, 1], bias [co], out NHWC tensor, out_coff, relu)."""
    n, h, w_, cbuf = x.shape
    ws = [m[0] for m in members]
    w_all = torch.cat(ws, dim=0)
    b_all = torch.cat([m[1].float().cpu() for m in members])
    wp, K, kpad = pack_weight(w_all)
    wp = wp.to(x.device)
    cout = w_all.shape[0]
    bias_p = torch.zeros(wp.shape[0], device=x.device, dtype=torch.float32)
    bias_p[:cout] = b_all.to(x.device)
    ho = (h - 1) // stride + 1
    wo = (w_ - 1) // stride + 1
    out0 = members[0][2]
    a = N.ConvArgs(x.data_ptr(), wp.data_ptr(), bias_p.data_ptr(), None, out0.data_ptr() + 2 * members[0][3],
                   n, h, w_, cbuf, cbuf, 1, 1, stride, stride, 0, 0, ho, wo, cout, K, kpad, out0.shape[-1], 0,
                   int(members[0][4]), 0, 1, 1)
    a.nseg = len(members)
    c0 = 0
    for s, (wt, b, out, coff, relu) in enumerate(members):
        a.seg_c0[s] = c0
        a.seg_ldy[s] = out.shape[-1]
        a.seg_relu[s] = int(relu)
        a.seg_y[s] = out.data_ptr() + 2 * coff
        c0 += wt.shape[0]
    L = N.lib()
    if cfg < 0:
        cfg = L.dml_conv_pick_cfg(C.byref(a))
    N.check(L.dml_conv(C.byref(a), cfg, N.stream_ptr()), "dml_conv(fused)")
    torch.cuda.current_stream().synchronize()
