"""ImageNet class index for top-5 decoding.

Keras' ``decode_predictions`` downloads ``imagenet_class_index.json`` (reference
models.py:42, 67). No network exists here and no copy of that file is present
(SURVEY §2.4), so a deterministic synthetic 1000-entry index is generated
("n%08d", "class_%04d"); a real index can be supplied by path
(``DML_CLASS_INDEX`` or ``load_class_index(path)``) in the same Keras JSON
format ``{"0": ["n01440764", "tench"], ...}``. The output format is unchanged.
"""
from __future__ import annotations

import json
import os
from functools import lru_cache
from typing import List, Optional, Tuple


def synthetic_index(classes: int = 1000) -> List[Tuple[str, str]]:
    return [(f"n{1000000 + 7919 * i:08d}", f"class_{i:04d}") for i in range(classes)]


@lru_cache(maxsize=4)
def load_class_index(path: Optional[str] = None, classes: int = 1000) -> Tuple[Tuple[str, str], ...]:
    path = path or os.environ.get("DML_CLASS_INDEX")
    if path and os.path.exists(path):
        with open(path) as f:
            d = json.load(f)
        return tuple(tuple(d[str(i)]) for i in range(len(d)))
    return tuple(synthetic_index(classes))
