"""Result files in the reference format.

Reference (worker.py:1580, models.py:42-44, 109-126, sample download/output_1_127.json):
file ``output_<job>_<batch>_<host.split('.')[0]>.json``, content
``{"<img>.jpeg": [[["<wnid>", "<label>", <prob>] x5]]}`` (outer list = Keras batch
dim, always 1), indent 4, numpy-safe; images that failed to download map to the
string "Failed to download file from SDFS" (worker.py:1382); ``get-output``
merges every ``output_<job>_*.json`` into ``final_<job>.json`` (worker.py:1496-1534).
"""
from __future__ import annotations

import ctypes as C
import json
import os
import threading
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from ..utils.labels import load_class_index

FAILED_DOWNLOAD = "Failed to download file from SDFS"
VERSION_SEP = "@"   # a store image pinned to one version: "<name>@<version>" (parallel/service.py)


class NpEncoder(json.JSONEncoder):
    def default(self, o):
        if isinstance(o, np.integer):
            return int(o)
        if isinstance(o, np.floating):
            return float(o)
        if isinstance(o, np.ndarray):
            return o.tolist()
        return super().default(o)


def image_key(name: str) -> str:
    """Output key of a batch image: its basename, without a pinned store version."""
    if "/" not in name and VERSION_SEP not in name:
        return name
    base = os.path.basename(name)
    head, sep, tail = base.rpartition(VERSION_SEP)
    return head if sep and tail.isdigit() else base


def output_name(job_id: int, batch_id: int, host: str) -> str:
    return f"output_{job_id}_{batch_id}_{host.split('.')[0].split(':')[0]}.json"


def decode_top5(names: Sequence[str], top_idx: np.ndarray, top_p: np.ndarray,
                failed: Iterable[str] = (), class_index=None) -> Dict[str, object]:
    """names[i] <- top-5 of row i, in decode_predictions format."""
    idx = class_index or load_class_index()
    out: Dict[str, object] = {}
    for i, name in enumerate(names):
        out[image_key(name)] = [[[idx[int(c)][0], idx[int(c)][1], float(p)]
                                 for c, p in zip(top_idx[i], top_p[i])]]
    for name in failed:
        out[image_key(name)] = FAILED_DOWNLOAD
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


# ----------------------------------------------------------- native renderer --
class BatchRenderer:
    """Renders a batch's output document byte-identically to
    ``dumps(decode_top5(...))`` in native code (csrc/host/output_json.cpp): the
    per-class text is pre-rendered once, image keys are cached, and the ctypes
    call releases the GIL, so a rank's writer thread does not stall its serve
    loop. Falls back to the Python encoder if the host library is unavailable."""

    def __init__(self, class_index=None):
        self.idx = class_index or load_class_index()
        self._keys: Dict[str, bytes] = {}
        self._lock = threading.Lock()
        self.lib = _host_lib()
        ind = " " * 16
        parts = [(json.dumps(w) + ",\n" + ind + json.dumps(lab) + ",\n" + ind).encode() for w, lab in self.idx]
        self.cls = b"".join(parts)
        off = np.zeros(len(parts) + 1, np.int64)
        np.cumsum([len(p) for p in parts], out=off[1:])
        self.cls_off = off
        self._tls = threading.local()   # per-thread scratch buffer: the ctypes call releases the GIL
        self.native = self.lib is not None

    def _key(self, name: str) -> bytes:
        k = self._keys.get(name)
        if k is None:
            base = image_key(name)
            # printable ASCII without quote / backslash: json.dumps adds the quotes only
            # (a job of unique synthetic names missed this cache for every image)
            k = (b'"' + base.encode() + b'"' if base.isascii() and base.isprintable() and '"' not in base
                 and "\\" not in base else json.dumps(base).encode())
            with self._lock:
                if len(self._keys) > 1 << 20:
                    self._keys.clear()
                self._keys[name] = k
        return k

    def render(self, images: Sequence[str], top_idx: np.ndarray, top_p: np.ndarray) -> bytes:
        """images[i] <- row i of top_idx/top_p ([n, 5]); a row whose first class
        id is negative is a failed image."""
        top_idx = np.ascontiguousarray(top_idx, dtype=np.int32)
        top_p = np.ascontiguousarray(top_p, dtype=np.float32)
        failed = top_idx[:, 0] < 0 if len(images) else np.zeros(0, bool)
        if not self.native:
            ok = [i for i in range(len(images)) if not failed[i]]
            doc = decode_top5([images[i] for i in ok], top_idx[ok], top_p[ok],
                              [images[i] for i in range(len(images)) if failed[i]], self.idx)
            return dumps(doc).encode()
        kc = self._keys
        names_k = [kc[nm] if nm in kc else self._key(nm) for nm in images]
        # decode_top5's dict: first-occurrence order, last assignment wins (a batch may repeat an
        # image: jobs pick cyclically); failed images are assigned after every decoded one
        if failed.any():
            fl = failed.tolist()
            ent: Dict[bytes, int] = {}
            for i, k in enumerate(names_k):
                if not fl[i]:
                    ent[k] = i
            for i, k in enumerate(names_k):
                if fl[i]:
                    ent[k] = -1
        else:
            ent = dict(zip(names_k, range(len(names_k))))
        keys = list(ent)
        rows = np.fromiter(ent.values(), np.int32, len(keys))
        koff = np.zeros(len(keys) + 1, np.int64)
        np.cumsum(np.fromiter(map(len, keys), np.int64, len(keys)), out=koff[1:])
        blob = b"".join(keys)
        k = top_idx.shape[1] if top_idx.ndim == 2 else 5
        need = 256 + len(blob) + len(keys) * k * 160
        buf = getattr(self._tls, "buf", None)
        if buf is None or C.sizeof(buf) < need:
            buf = self._tls.buf = C.create_string_buffer(max(need, 1 << 20))
        n = self.lib.dml_render_top5_json(len(keys), blob, koff.ctypes.data, rows.ctypes.data, top_idx.ctypes.data,
                                          top_p.ctypes.data, k, self.cls, self.cls_off.ctypes.data, len(self.idx),
                                          buf, C.sizeof(buf))
        if n < 0:
            raise RuntimeError("output render buffer too small")
        return C.string_at(buf, n)   # copies n bytes (buf.raw copied the whole 1 MiB scratch first)


    def render_merged(self, batches: Sequence[Tuple[Sequence[str], np.ndarray, np.ndarray]]) -> bytes:
        """final_<job>.json straight from the batches' top-5 rows (images, ids [n, 5], probs
        [n, 5]; ids[i, 0] < 0 = failed), in the order get-output merges their files:
        byte-identical to ``json.dump(merge_outputs([doc(b) for b in batches]), indent=4)``
        where doc(b) is the batch's own output document (decoded images first, then the
        failed ones; dict update keeps a key's first position, the last value wins)."""
        if not batches:
            return b"{}"
        if not self.native:
            docs = []
            for names, ids, probs in batches:
                bad = ids[:, 0] < 0
                ok = [i for i in range(len(names)) if not bad[i]]
                docs.append(decode_top5([names[i] for i in ok], ids[ok], probs[ok],
                                        [names[i] for i in range(len(names)) if bad[i]], self.idx))
            return dumps(merge_outputs(docs)).encode()
        kc = self._keys
        merged: Dict[bytes, int] = {}
        off = 0
        for names, ids, _ in batches:
            keys = [kc[nm] if nm in kc else self._key(nm) for nm in names]
            fl = (np.asarray(ids)[:, 0] < 0).tolist() if len(names) else []
            ent: Dict[bytes, int] = {}
            for i, k in enumerate(keys):
                if not fl[i]:
                    ent[k] = off + i
            for i, k in enumerate(keys):
                if fl[i]:
                    ent[k] = -1
            merged.update(ent)
            off += len(names)
        top_idx = np.ascontiguousarray(np.concatenate([np.asarray(b[1], np.int32) for b in batches]), np.int32)
        top_p = np.ascontiguousarray(np.concatenate([np.asarray(b[2], np.float32) for b in batches]), np.float32)
        keys = list(merged)
        rows = np.fromiter(merged.values(), np.int32, len(keys))
        koff = np.zeros(len(keys) + 1, np.int64)
        np.cumsum(np.fromiter(map(len, keys), np.int64, len(keys)), out=koff[1:])
        blob = b"".join(keys)
        need = 256 + len(blob) + len(keys) * 5 * 160
        buf = C.create_string_buffer(need)
        n = self.lib.dml_render_top5_json(len(keys), blob, koff.ctypes.data, rows.ctypes.data, top_idx.ctypes.data,
                                          top_p.ctypes.data, 5, self.cls, self.cls_off.ctypes.data, len(self.idx),
                                          buf, need)
        if n < 0:
            raise RuntimeError("final output render buffer too small")
        return C.string_at(buf, n)


_host = None
_host_lock = threading.Lock()


def _host_lib():
    """libdml_host.so (built with g++ on first use; None if no compiler and no library)."""
    global _host
    if _host is not None:
        return _host or None
    with _host_lock:
        if _host is None:
            from .. import _build

            try:
                path = _build.build_host() if os.environ.get("DML_SKIP_BUILD") != "1" else _build.HOST_LIB_PATH
                L = C.CDLL(str(path))
                L.dml_render_top5_json.restype = C.c_long
                L.dml_render_top5_json.argtypes = [C.c_int, C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                   C.c_void_p, C.c_int, C.c_char_p, C.c_void_p, C.c_int, C.c_void_p,
                                                   C.c_long]
                L.dml_py_repr.restype = C.c_int
                L.dml_py_repr.argtypes = [C.c_double, C.c_char_p]
                _host = L
            except Exception:  # no compiler and no shipped library: Python encoder
                _host = False
    return _host or None
