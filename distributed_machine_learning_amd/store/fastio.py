"""Batched file operations of the store's same-node path (csrc/host/store_io.cpp).

A bundle's spool files and a replica's hard links are made by ONE native call each, with the
GIL released once, instead of one Python syscall (and one GIL re-acquisition behind the
rank's other threads) per file. Falls back to plain Python when libdml_host.so is missing.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Sequence, Tuple

_fns = None


def _lib():
    global _fns
    if _fns is None:
        from ..serving.output import _host_lib

        L = _host_lib()
        if L is None or not hasattr(L, "dml_link_many"):
            _fns = False
        else:
            L.dml_spool_write.restype = C.c_int
            L.dml_spool_write.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                          C.POINTER(C.c_long)]
            L.dml_link_many.restype = C.c_int
            L.dml_link_many.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.POINTER(C.c_int)]
            if hasattr(L, "dml_read_many"):
                L.dml_read_many.restype = C.c_long
                L.dml_read_many.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.c_void_p, C.c_long,
                                            C.POINTER(C.c_long), C.POINTER(C.c_long)]
            _fns = L
    return _fns or None


def spool_write(d: str, items: Sequence[Tuple[str, bytes]]) -> None:
    """dir d (created) <- one file per (name, bytes)."""
    for name, _ in items:
        if "/" in name or name.startswith(".."):
            raise ValueError(f"bad sdfs name {name!r}")
    L = _lib()
    if L is None:
        os.makedirs(d, exist_ok=True)
        for name, data in items:
            with open(os.path.join(d, name), "wb") as f:
                f.write(data)
        return
    n = len(items)
    names = (C.c_char_p * n)(*[nm.encode() for nm, _ in items])
    datas = (C.c_char_p * n)(*[data for _, data in items])
    lens = (C.c_long * n)(*[len(data) for _, data in items])
    rc = L.dml_spool_write(d.encode(), n, names, datas, lens)
    if rc != 0:
        raise OSError(-rc, os.strerror(-rc), d)


def link_many(pairs: Sequence[Tuple[str, str]]) -> List[int]:
    """dst <- hard link of src for each (src, dst), replacing dst atomically; per pair 0 or
    -errno."""
    L = _lib()
    if L is None:
        out = []
        for src, dst in pairs:
            tmp = dst + ".lnk"
            try:
                try:
                    os.remove(tmp)
                except FileNotFoundError:
                    pass
                os.link(src, tmp)
                os.replace(tmp, dst)
                out.append(0)
            except OSError as e:
                out.append(-(e.errno or 1))
        return out
    n = len(pairs)
    srcs = (C.c_char_p * n)(*[s.encode() for s, _ in pairs])
    dsts = (C.c_char_p * n)(*[d.encode() for _, d in pairs])
    st = (C.c_int * n)()
    L.dml_link_many(n, srcs, dsts, st)
    return list(st)


def read_many(paths: Sequence[str]) -> List[memoryview]:
    """The whole contents of each file (one buffer, a memoryview per file): two native calls
    (sizes, then bytes), the GIL released in each. Raises OSError like open()."""
    L = _lib()
    if L is None or not hasattr(L, "dml_read_many"):
        out = []
        for p in paths:
            with open(p, "rb") as f:
                out.append(memoryview(f.read()))
        return out
    n = len(paths)
    ps = (C.c_char_p * n)(*[p.encode() for p in paths])
    offs = (C.c_long * n)()
    lens = (C.c_long * n)()
    total = L.dml_read_many(n, ps, None, 0, offs, lens)
    if total < 0:
        raise OSError(-total, os.strerror(-total))
    buf = bytearray(max(total, 1))
    cbuf = (C.c_char * len(buf)).from_buffer(buf)
    got = L.dml_read_many(n, ps, C.addressof(cbuf), len(buf), offs, lens)
    del cbuf
    if got < 0:
        raise OSError(-got, os.strerror(-got))
    mv = memoryview(buf)
    return [mv[offs[i]:offs[i] + lens[i]] for i in range(n)]
