"""Model zoo: the two classifiers the reference serves (models.py:23-71)."""
from __future__ import annotations

from typing import Tuple

from .graph import Graph
from .inception_v3 import build_inception_v3
from .resnet50 import build_resnet50
from .weights import Weights, init_weights

MODELS = {"ResNet50": build_resnet50, "InceptionV3": build_inception_v3}
_ALIASES = {"resnet50": "ResNet50", "resnet": "ResNet50", "inceptionv3": "InceptionV3", "inception": "InceptionV3",
            "inception_v3": "InceptionV3"}


def canonical_name(name: str) -> str:
    if name in MODELS:
        return name
    key = name.lower()
    if key in _ALIASES:
        return _ALIASES[key]
    raise KeyError(f"unknown model {name!r}; choose from {sorted(MODELS)}")


def build_graph(name: str) -> Graph:
    return MODELS[canonical_name(name)]()


def build_model(name: str, seed: int = 0, calibrate: bool = True, calib_batch: int = 32) -> Tuple[Graph, Weights]:
    """Graph + deterministic random-init weights (optionally BN-calibrated on
    synthetic images so activations stay normalised through the depth)."""
    g = build_graph(name)
    w = init_weights(g, seed)
    if calibrate:
        import torch

        from .oracle import calibrate_bn, preprocess_reference

        gen = torch.Generator().manual_seed(seed + 1234)
        hw = g.input_hw
        imgs = torch.randint(0, 256, (calib_batch, hw[0], hw[1], 3), dtype=torch.uint8, generator=gen)
        w = calibrate_bn(g, w, preprocess_reference(imgs, hw, g.preprocess))
    return g, w


__all__ = ["Graph", "Weights", "MODELS", "build_graph", "build_model", "canonical_name", "init_weights"]
