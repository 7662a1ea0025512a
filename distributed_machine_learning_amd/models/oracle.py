"""Plain-PyTorch fp32 executor of the layer IR — the numerics oracle.

Runs NCHW on any device (CPU in tests) with BatchNorm applied UNFUSED from its
raw statistics, so a bug in the engine's BN folding, channel-offset concat,
implicit-GEMM padding or pooling divisor shows up as a mismatch. Also provides
the preprocessing oracle (Pillow-NEAREST resize + caffe/tf normalisation,
reference models.py:34-38 / 59-63).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

from .graph import Conv, Dense, FusedConv, Graph, GlobalAvgPool, Pool
from .weights import Weights

CAFFE_MEAN_BGR = (103.939, 116.779, 123.68)


def preprocess_reference(images_u8: torch.Tensor, out_hw, mode: str) -> torch.Tensor:
    """uint8 [N, Hs, Ws, 3] RGB -> fp32 NCHW [N, 3, Ho, Wo]."""
    n, hs, ws, _ = images_u8.shape
    ho, wo = out_hw
    iy = torch.clamp(((torch.arange(ho, dtype=torch.float32) + 0.5) * (hs / ho)).floor().long(), max=hs - 1)
    ix = torch.clamp(((torch.arange(wo, dtype=torch.float32) + 0.5) * (ws / wo)).floor().long(), max=ws - 1)
    x = images_u8[:, iy][:, :, ix].float()  # N, Ho, Wo, 3 (RGB)
    if mode == "caffe":
        x = x[..., [2, 1, 0]] - torch.tensor(CAFFE_MEAN_BGR)
    else:
        x = x / 127.5 - 1.0
    return x.permute(0, 3, 1, 2).contiguous()


def _bf16(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.bfloat16).to(x.dtype)


class OracleExecutor:
    """fp32 reference. With ``emulate_bf16=True`` it reproduces the engine's
    rounding points instead (BN folded, weights and every stored activation
    rounded to bf16, fp32 accumulation) — the tight reference for whole-network
    tests, since random-init deep nets amplify bf16 rounding chaotically."""

    def __init__(self, g: Graph, w: Weights, device="cpu", dtype=torch.float32, emulate_bf16: bool = False):
        self.g, self.device, self.dtype = g, device, dtype
        self.emulate = emulate_bf16
        self.p = {k: torch.from_numpy(np.ascontiguousarray(v)).to(device, dtype) for k, v in w.items()}
        if emulate_bf16:
            from .weights import fold_conv

            self.folded = {}
            for n in g.nodes:
                for c in (n.members if isinstance(n, FusedConv) else ([n] if isinstance(n, Conv) else [])):
                    k, b = fold_conv(c, w)
                    self.folded[c.name] = (_bf16(torch.from_numpy(k).permute(3, 2, 0, 1).to(device, dtype)),
                                           torch.from_numpy(b).to(device, dtype))
                if isinstance(n, Dense):
                    self.folded[n.name] = (_bf16(self.p[f"{n.name}/kernel"]), self.p[f"{n.name}/bias"])

    def _bn(self, n: Conv, y: torch.Tensor) -> torch.Tensor:
        p = self.p
        gamma = p.get(f"{n.name}/gamma")
        mean, var, beta = p[f"{n.name}/mean"], p[f"{n.name}/var"], p[f"{n.name}/beta"]
        y = (y - mean[None, :, None, None]) / torch.sqrt(var[None, :, None, None] + n.bn_eps)
        if gamma is not None:
            y = y * gamma[None, :, None, None]
        return y + beta[None, :, None, None]

    @torch.no_grad()
    def forward(self, x: torch.Tensor, keep: bool = False) -> Dict[str, torch.Tensor]:
        """x: preprocessed NCHW fp32. Returns tensors dict (logits, probs, and all if keep)."""
        g, p = self.g, self.p
        n_img = x.shape[0]
        em = self.emulate
        rnd = _bf16 if em else (lambda v: v)
        t: Dict[str, torch.Tensor] = {g.input: rnd(x.to(self.device, self.dtype))}
        for n in g.nodes:
            convs = n.members if isinstance(n, FusedConv) else ([n] if isinstance(n, Conv) else [])
            for c in convs:
                src = t[c.inp][:, c.in_coff:c.in_coff + c.cin]
                if em:
                    k, b = self.folded[c.name]
                    y = F.conv2d(src, k, b, stride=(c.sh, c.sw), padding=(c.ph, c.pw))
                else:
                    k = p[f"{c.name}/kernel"].permute(3, 2, 0, 1)  # HWIO -> OIHW
                    y = F.conv2d(src, k, p.get(f"{c.name}/bias"), stride=(c.sh, c.sw), padding=(c.ph, c.pw))
                    if c.bn:
                        y = self._bn(c, y)
                if c.residual:
                    y = y + t[c.residual][:, :, ::c.res_sub, ::c.res_sub]
                if c.relu:
                    y = F.relu(y)
                self._write(t, c.out, rnd(y), c.out_coff, n_img)
            if isinstance(n, Pool):
                src = t[n.inp]
                if n.mode == "max":
                    y = F.max_pool2d(F.pad(src, (n.pad,) * 4), n.k, n.stride)  # Keras ZeroPadding2D + valid pool
                else:
                    y = F.avg_pool2d(src, n.k, n.stride, padding=n.pad, count_include_pad=False)
                if n.relu:
                    y = F.relu(y)
                self._write(t, n.out, rnd(y), n.out_coff, n_img)
            elif isinstance(n, GlobalAvgPool):
                t[n.out] = rnd(t[n.inp].mean(dim=(2, 3), keepdim=True))
            elif isinstance(n, Dense):
                if em:
                    k, b = self.folded[n.name]
                    y = t[n.inp].flatten(1) @ k + b
                else:
                    y = t[n.inp].flatten(1) @ p[f"{n.name}/kernel"] + p[f"{n.name}/bias"]
                t[n.out] = y
        out = {"logits": t[g.logits], "probs": torch.softmax(t[g.logits], dim=-1)}
        if keep:
            out.update(t)
        return out

    def _write(self, t, name, y, coff, n_img):
        h, w, c = self.g.shape(name)
        if coff == 0 and y.shape[1] == c:
            t[name] = y
            return
        if name not in t:
            t[name] = torch.zeros((n_img, c, h, w), device=y.device, dtype=y.dtype)
        t[name][:, coff:coff + y.shape[1]] = y


def synthetic_images(n: int, hw, seed: int = 0, noise: float = 24.0) -> torch.Tensor:
    """uint8 [n, H, W, 3] test images with image-level structure: a random base
    colour, four random low-frequency colour gratings and pixel noise. IID
    uniform noise images all have the same statistics, so a random-init
    network's pooled features (and logits) barely depend on them; these differ
    image to image the way natural photos do, which makes a numerics check
    input-sensitive (models/weights.py 'head calibration')."""
    rng = np.random.default_rng(seed)
    H, W = hw
    yy, xx = np.meshgrid(np.linspace(0.0, 1.0, H), np.linspace(0.0, 1.0, W), indexing="ij")
    out = np.empty((n, H, W, 3), np.uint8)
    for i in range(n):
        img = np.zeros((H, W, 3)) + rng.uniform(40, 215, 3)
        for _ in range(4):
            fx, fy = rng.uniform(0.5, 6.0, 2)
            ph = rng.uniform(0.0, 2 * np.pi)
            amp = rng.uniform(10, 50, 3)
            img += amp * np.sin(2 * np.pi * (fx * xx + fy * yy) + ph)[..., None]
        img += rng.uniform(-noise, noise, (H, W, 3))
        out[i] = np.clip(img, 0, 255).astype(np.uint8)
    return torch.from_numpy(out)


@torch.no_grad()
def calibrate_head(g: Graph, w: Weights, x: torch.Tensor, scale: float = 3.0) -> Weights:
    """Per-class standardisation of the classifier over the calibration batch:
    logit_c <- (logit_c - mean_c) * scale / std_c (folded into the Dense kernel
    and bias). A trained classifier's logits vary with the image by several
    units per class; a random-init head's vary by a small fraction of a large
    common offset, so top-1 would be the same class for every image."""
    dense = [n for n in g.nodes if isinstance(n, Dense)]
    if not dense:
        return w
    d = dense[-1]
    out = OracleExecutor(g, w).forward(x, keep=True)
    f = out[d.inp].flatten(1)
    k = torch.from_numpy(w[f"{d.name}/kernel"]).float()
    b = torch.from_numpy(w[f"{d.name}/bias"]).float()
    z = f @ k + b
    mu, sd = z.mean(0), z.std(0).clamp_min(1e-6)
    w = dict(w)
    w[f"{d.name}/kernel"] = (k * (scale / sd)).numpy().astype(np.float32)
    w[f"{d.name}/bias"] = ((b - mu) * (scale / sd)).numpy().astype(np.float32)
    return w


@torch.no_grad()
def calibrate_bn(g: Graph, w: Weights, x: torch.Tensor) -> Weights:
    """Set every BN's mean/var to the batch statistics of its conv output on x
    (data-dependent init), so activations stay normalised through the depth."""
    w = dict(w)
    ex = OracleExecutor(g, w)
    p = ex.p
    n_img = x.shape[0]
    t = {g.input: x.float()}
    for n in g.nodes:
        if isinstance(n, Conv):
            src = t[n.inp][:, n.in_coff:n.in_coff + n.cin]
            k = p[f"{n.name}/kernel"].permute(3, 2, 0, 1)
            y = F.conv2d(src, k, p.get(f"{n.name}/bias"), stride=(n.sh, n.sw), padding=(n.ph, n.pw))
            if n.bn:
                mean = y.mean(dim=(0, 2, 3))
                var = y.var(dim=(0, 2, 3), unbiased=False)
                w[f"{n.name}/mean"] = mean.numpy().astype(np.float32)
                w[f"{n.name}/var"] = var.numpy().astype(np.float32)
                p[f"{n.name}/mean"], p[f"{n.name}/var"] = mean, var
                y = ex._bn(n, y)
            if n.residual:
                y = y + t[n.residual][:, :, ::n.res_sub, ::n.res_sub]
            if n.relu:
                y = F.relu(y)
            ex._write(t, n.out, y, n.out_coff, n_img)
        elif isinstance(n, Pool):
            src = t[n.inp]
            if n.mode == "max":
                y = F.max_pool2d(F.pad(src, (n.pad,) * 4), n.k, n.stride)
            else:
                y = F.avg_pool2d(src, n.k, n.stride, padding=n.pad, count_include_pad=False)
            ex._write(t, n.out, y, n.out_coff, n_img)
        elif isinstance(n, GlobalAvgPool):
            t[n.out] = t[n.inp].mean(dim=(2, 3), keepdim=True)
        elif isinstance(n, Dense):
            t[n.out] = t[n.inp].flatten(1) @ p[f"{n.name}/kernel"] + p[f"{n.name}/bias"]
    return w
