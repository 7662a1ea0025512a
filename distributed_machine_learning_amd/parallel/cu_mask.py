"""CU-masked HIP streams: give each concurrent sub-batch its own share of the chip.

By default the two sub-batch streams of a ``SplitEngine`` (the pipeline's compute
stream and one extra stream) both dispatch over all 256 CUs, so at any moment
an XCD's L2 serves the working sets of two unrelated layers. With
``DML_CU_MASK=<pattern>`` the pipeline's compute stream (part 0) and the
SplitEngine's extra stream (part 1) are created by
``hipExtStreamCreateWithCUMask`` (``dml_stream_create_cu_mask``) over
complementary halves of the CUs:

* ``lohi``    logical CUs [0, n/2) / [n/2, n)
* ``mod8``    logical CU i to part (i % 8) // 4
* ``evenodd`` logical CU i to part i % 2
* ``0x..,0x..;0x..,..``  explicit 32-bit mask words of part 0 ; part 1

Which of these keeps a sub-batch on whole XCDs depends on how the runtime numbers
logical CUs; ``tools/gpu_cumask.sh`` measures all of them.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional

import torch

from .. import _native as N

PARTS = 2


def num_cus() -> int:
    cus, ma, mi = C.c_int(), C.c_int(), C.c_int()
    N.check(N.lib().dml_device_info(C.byref(cus), C.byref(ma), C.byref(mi)), "device info")
    return cus.value


def mask_words(pattern: str, part: int, ncu: int) -> List[int]:
    """The 32-bit mask words of ``part`` (0 or 1) for a named or explicit pattern."""
    if not 0 <= part < PARTS:
        raise ValueError(f"part {part} not in [0, {PARTS})")
    nwords = (ncu + 31) // 32
    if pattern.startswith("0x"):
        parts = pattern.split(";")
        if len(parts) != PARTS:
            raise ValueError("explicit DML_CU_MASK needs one word list per part, ';'-separated")
        words = [int(w, 16) for w in parts[part].split(",")]
        if len(words) != nwords:
            raise ValueError(f"explicit mask needs {nwords} words, got {len(words)}")
        return words
    if pattern == "lohi":
        sel = [part == (i * PARTS) // ncu for i in range(ncu)]
    elif pattern == "mod8":
        sel = [part == (i % 8) * PARTS // 8 for i in range(ncu)]
    elif pattern == "evenodd":
        sel = [part == i % PARTS for i in range(ncu)]
    else:
        raise ValueError(f"unknown CU mask pattern {pattern!r}")
    words = [0] * nwords
    for i, on in enumerate(sel):
        if on:
            words[i // 32] |= 1 << (i % 32)
    return words


class MaskedStream:
    """A HIP stream restricted to the CUs of ``words`` (owned; destroyed with
    this object), usable wherever a torch stream is (``.stream``)."""

    def __init__(self, device: torch.device, words: List[int]):
        self.words = list(words)
        arr = (C.c_uint * len(words))(*words)
        h = C.c_void_p()
        with torch.cuda.device(device):
            N.check(N.lib().dml_stream_create_cu_mask(arr, len(words), C.byref(h)), "CU-masked stream")
        self.handle = h
        self.stream = torch.cuda.ExternalStream(h.value, device=device)

    def __del__(self):
        try:
            if self.handle:
                N.lib().dml_stream_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


def from_env(device: torch.device, part: int) -> Optional[MaskedStream]:
    """A masked stream for ``part`` when ``DML_CU_MASK`` is set, else None."""
    pattern = os.environ.get("DML_CU_MASK", "")
    if not pattern or torch.device(device).type != "cuda":
        return None
    return MaskedStream(torch.device(device), mask_words(pattern, part, num_cus()))
