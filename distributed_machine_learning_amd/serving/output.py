"""Result files in the reference format.

Reference (worker.py:1580, models.py:42-44, 109-126, sample download/output_1_127.json):
file ``output_<job>_<batch>_<host.split('.')[0]>.json``, content
``{"<img>.jpeg": [[["<wnid>", "<label>", <prob>] x5]]}`` (outer list = Keras batch
dim, always 1), indent 4, numpy-safe; images that failed to download map to the
string "Failed to download file from SDFS" (worker.py:1382); ``get-output``
merges every ``output_<job>_*.json`` into ``final_<job>.json`` (worker.py:1496-1534).
"""
from __future__ import annotations

import json
import os
from typing import Dict, Iterable, Sequence

import numpy as np

from ..utils.labels import load_class_index

FAILED_DOWNLOAD = "Failed to download file from SDFS"


class NpEncoder(json.JSONEncoder):
    def default(self, o):
        if isinstance(o, np.integer):
            return int(o)
        if isinstance(o, np.floating):
            return float(o)
        if isinstance(o, np.ndarray):
            return o.tolist()
        return super().default(o)


def output_name(job_id: int, batch_id: int, host: str) -> str:
    return f"output_{job_id}_{batch_id}_{host.split('.')[0].split(':')[0]}.json"


def decode_top5(names: Sequence[str], top_idx: np.ndarray, top_p: np.ndarray,
                failed: Iterable[str] = (), class_index=None) -> Dict[str, object]:
    """names[i] <- top-5 of row i, in decode_predictions format."""
    idx = class_index or load_class_index()
    out: Dict[str, object] = {}
    for i, name in enumerate(names):
        out[os.path.basename(name)] = [[[idx[int(c)][0], idx[int(c)][1], float(p)]
                                        for c, p in zip(top_idx[i], top_p[i])]]
    for name in failed:
        out[os.path.basename(name)] = FAILED_DOWNLOAD
    return out


def dumps(result: Dict[str, object]) -> str:
    return json.dumps(result, indent=4, cls=NpEncoder)


def write_output(path: str, result: Dict[str, object]) -> str:
    with open(path, "w") as f:
        f.write(dumps(result))
    return path


def merge_outputs(docs: Iterable[Dict[str, object]]) -> Dict[str, object]:
    merged: Dict[str, object] = {}
    for d in docs:
        merged.update(d)
    return merged
