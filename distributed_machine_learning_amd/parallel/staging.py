"""Host-pinned image arena + async host->HBM staging (per worker process).

Replaces the reference's data path — scp of every image from an SDFS replica
to the worker's disk, then a PIL read (worker.py:1365-1366,
file_service.py:116-124, models.py:34/59) — with one pinned (hipHostMalloc)
arena per worker holding uint8 HWC images, and hipMemcpyAsync of a whole batch
on a dedicated copy stream, double-buffered against the compute stream.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import _native as N


class PinnedImageStore:
    """A fixed-shape uint8 image arena in pinned host memory: [capacity, H, W, 3]."""

    def __init__(self, capacity: int, hw=(224, 224)):
        self.capacity, self.hw = capacity, tuple(hw)
        self.img_bytes = hw[0] * hw[1] * 3
        self.nbytes = capacity * self.img_bytes
        self.lib = N.lib()
        self.ptr = self.lib.dml_host_alloc(self.nbytes)
        if not self.ptr:
            raise N.NativeError("pinned alloc failed: " + self.lib.dml_last_error().decode())
        buf = (C.c_uint8 * self.nbytes).from_address(self.ptr)
        self.array = np.frombuffer(buf, dtype=np.uint8).reshape(capacity, hw[0], hw[1], 3)
        self.names: List[Optional[str]] = [None] * capacity

    def fill_synthetic(self, seed: int = 0) -> None:
        rng = np.random.default_rng(seed)
        # write in chunks (avoid a second full-size temporary)
        for i in range(0, self.capacity, 64):
            j = min(self.capacity, i + 64)
            self.array[i:j] = rng.integers(0, 256, size=(j - i, *self.hw, 3), dtype=np.uint8)
            for k in range(i, j):
                self.names[k] = f"synthetic_{seed}_{k}.jpeg"

    def put(self, index: int, img_u8: np.ndarray, name: str) -> None:
        assert img_u8.shape == (*self.hw, 3) and img_u8.dtype == np.uint8
        self.array[index] = img_u8
        self.names[index] = name

    def h2d(self, dst: torch.Tensor, start: int, count: int, stream: torch.cuda.Stream) -> None:
        """Async copy images [start, start+count) (wrapping) into dst[:count] on `stream`."""
        assert dst.dtype == torch.uint8 and dst.is_contiguous()
        done = 0
        while done < count:
            s = (start + done) % self.capacity
            n = min(count - done, self.capacity - s)
            N.check(self.lib.dml_memcpy_h2d_async(dst.data_ptr() + done * self.img_bytes,
                                                  self.ptr + s * self.img_bytes, n * self.img_bytes,
                                                  N.stream_ptr(stream)), "h2d")
            done += n

    def h2d_indices(self, dst: torch.Tensor, indices: Sequence[int], stream: torch.cuda.Stream) -> None:
        """Gather arbitrary images (coalescing contiguous runs into one copy each)."""
        i = 0
        idx = list(indices)
        while i < len(idx):
            j = i + 1
            while j < len(idx) and idx[j] == idx[j - 1] + 1:
                j += 1
            N.check(self.lib.dml_memcpy_h2d_async(dst.data_ptr() + i * self.img_bytes,
                                                  self.ptr + idx[i] * self.img_bytes, (j - i) * self.img_bytes,
                                                  N.stream_ptr(stream)), "h2d")
            i = j

    def close(self) -> None:
        if getattr(self, "ptr", None):
            self.array = None
            self.lib.dml_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
