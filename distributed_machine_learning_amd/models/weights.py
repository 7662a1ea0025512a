"""Deterministic random-init weights, BatchNorm folding and (de)serialisation.

The reference downloads ImageNet weights through Keras (models.py:26,51); no
network exists here, so weights are generated from a seed (He-normal kernels,
BatchNorm statistics optionally calibrated on synthetic images so activations
stay O(1) through the depth like a trained net's). Storage format: safetensors
(no pickle anywhere), keys ``<layer>/kernel`` (Keras HWIO), ``<layer>/bias``,
``<layer>/gamma|beta|mean|var``.
"""
from __future__ import annotations

from typing import Dict

import numpy as np

from .graph import Conv, Dense, Graph

Weights = Dict[str, np.ndarray]


# Numerically well-conditioned random init. A random-init deep ReLU net with
# per-channel normalisation is chaotic: bf16 rounding at every layer is amplified
# through the depth (fp32 vs bf16-emulated logits differed by 12 % / 20 % max-rel
# on ResNet50 / InceptionV3 with the plain init, top-1 agreement 81 % / 63 %),
# which made any whole-network numerics check loose. Two standard remedies:
#  * residual nets: the BN gamma of each residual branch's last conv is scaled
#    by RES_GAMMA (the "zero-gamma" residual init of Goyal et al., 2017): the
#    identity path dominates -> ResNet50 gap 0.4 %, top-5 identical;
#  * nets without residuals (InceptionV3, BN without scale): BN beta shifted by
#    BETA_SHIFT before calibration, so ReLUs operate mostly in their linear
#    region -> InceptionV3 gap 3.6 %, top-1 identical, top-5 overlap >= 4/5
#    (32 images; /tmp experiment recorded in DESIGN.md §3 "Numerics").
RES_GAMMA = 0.12
BETA_SHIFT = 1.0


def init_weights(g: Graph, seed: int = 0) -> Weights:
    rng = np.random.default_rng(seed)
    w: Weights = {}
    residual_net = any(isinstance(n, Conv) and n.residual for n in g.nodes)
    for n in g.nodes:
        if isinstance(n, Conv):
            fan_in = n.kh * n.kw * n.cin
            w[f"{n.name}/kernel"] = (rng.standard_normal((n.kh, n.kw, n.cin, n.cout)) * np.sqrt(2.0 / fan_in)).astype(np.float32)
            if n.bias:
                w[f"{n.name}/bias"] = (rng.standard_normal(n.cout) * 0.05).astype(np.float32)
            if n.bn:
                if n.bn_scale:
                    gam = rng.uniform(0.8, 1.2, n.cout)
                    if n.residual:  # last conv of a residual branch
                        gam = gam * RES_GAMMA
                    w[f"{n.name}/gamma"] = gam.astype(np.float32)
                beta = rng.standard_normal(n.cout) * 0.1
                if not residual_net:
                    beta = beta + BETA_SHIFT
                w[f"{n.name}/beta"] = beta.astype(np.float32)
                w[f"{n.name}/mean"] = (rng.standard_normal(n.cout) * 0.1).astype(np.float32)
                w[f"{n.name}/var"] = rng.uniform(0.5, 1.5, n.cout).astype(np.float32)
        elif isinstance(n, Dense):
            w[f"{n.name}/kernel"] = (rng.standard_normal((n.cin, n.cout)) * np.sqrt(1.0 / n.cin)).astype(np.float32)
            w[f"{n.name}/bias"] = (rng.standard_normal(n.cout) * 0.01).astype(np.float32)
    return w


def fold_conv(n: Conv, w: Weights):
    """Return (kernel HWIO fp32, bias fp32) with BatchNorm folded in:
    k' = k * gamma / sqrt(var + eps);  b' = (b - mean) * gamma / sqrt(var + eps) + beta."""
    k = w[f"{n.name}/kernel"].astype(np.float64)
    b = w.get(f"{n.name}/bias")
    b = np.zeros(n.cout) if b is None else b.astype(np.float64)
    if n.bn:
        gamma = w.get(f"{n.name}/gamma")
        gamma = np.ones(n.cout) if gamma is None else gamma.astype(np.float64)
        scale = gamma / np.sqrt(w[f"{n.name}/var"].astype(np.float64) + n.bn_eps)
        k = k * scale
        b = (b - w[f"{n.name}/mean"]) * scale + w[f"{n.name}/beta"]
    return k.astype(np.float32), b.astype(np.float32)


def save_weights(path: str, w: Weights) -> None:
    from safetensors.numpy import save_file

    save_file({k: np.ascontiguousarray(v) for k, v in w.items()}, path)


def load_weights(path: str) -> Weights:
    from safetensors.numpy import load_file

    return dict(load_file(path))
