"""JPEG decode worker processes for the store-image path (GpuRankBackend).

Why processes: in the rank process a decode is ~0.8 ms of Pillow C code (GIL released) plus
~0.3 ms of `tobytes` / array conversion and Python bookkeeping that holds the GIL, so 32 decode
threads topped out at ~3.5k images/s on the 51,200-distinct run while competing with the serve
loop for the GIL. Each worker is a plain child process (`python -m ...decode_worker`: numpy /
Pillow only — no torch, no GPU) fed over its stdin/stdout pipes: the rank's pool thread writes a
chunk of JPEG bytes and reads back the RGB rows, both syscalls with the GIL released.

Protocol (little endian): request = u32 n, then n x (u32 len, bytes); reply = n x (i32 h, i32 w,
h*w*3 bytes of RGB), h = -1 for an undecodable file. Decode semantics = Keras load_img's (and
serving.inference.load_image's): Image.open, convert("RGB") unless already RGB.
"""
from __future__ import annotations

import io
import os
import queue
import struct
import subprocess
import sys
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np


def _read_exact(f, n: int) -> bytes:
    """n bytes from a pipe (an unbuffered read returns what is there: loop)."""
    parts, got = [], 0
    while got < n:
        b = f.read(n - got)
        if not b:
            raise EOFError("decode worker pipe closed")
        parts.append(b)
        got += len(b)
    return parts[0] if len(parts) == 1 else b"".join(parts)


def _serve() -> None:
    from PIL import Image

    rd, wr = sys.stdin.buffer, sys.stdout.buffer
    while True:
        hdr = rd.read(4)
        if not hdr or len(hdr) < 4:
            return
        (n,) = struct.unpack("<I", hdr)
        out = []
        for _ in range(n):
            (ln,) = struct.unpack("<I", _read_exact(rd, 4))
            data = _read_exact(rd, ln)
            try:
                im = Image.open(io.BytesIO(data))
                if im.mode != "RGB":
                    im = im.convert("RGB")
                raw = im.tobytes()
                out.append(struct.pack("<ii", im.height, im.width))
                out.append(raw)
            except Exception:  # undecodable: reported as failed, the worker lives on
                out.append(struct.pack("<ii", -1, -1))
        wr.write(b"".join(out))
        wr.flush()


class DecodeProcs:
    """N worker processes; `decode_many` hands one chunk to a free worker (blocking while all
    are busy) and returns {name: RGB array or None}. Thread-safe; workers end with the rank
    (stdin EOF)."""

    def __init__(self, n: int):
        env = dict(os.environ, OMP_NUM_THREADS="1")
        cmd = [sys.executable, "-m", "distributed_machine_learning_amd.parallel.decode_worker"]
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        self._cmd, self._env = cmd, env
        self.procs = [self._spawn() for _ in range(max(1, n))]
        self.free: "queue.Queue[subprocess.Popen]" = queue.Queue()
        for p in self.procs:
            self.free.put(p)
        self._lock = threading.Lock()
        self.closed = False
        self.get_timeout_s = 30.0

    def _spawn(self) -> subprocess.Popen:
        p = subprocess.Popen(self._cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, env=self._env, bufsize=0)
        if hasattr(self, "procs"):
            self.procs.append(p)
        return p

    def decode_many(self, items: Sequence[Tuple[str, bytes]]) -> Dict[str, Optional[np.ndarray]]:
        if not items:
            return {}
        try:
            p = self.free.get(timeout=self.get_timeout_s)
        except queue.Empty:
            raise TimeoutError("no decode worker free") from None   # the caller decodes in-process
        try:
            req = [struct.pack("<I", len(items))]
            for _, data in items:
                req.append(struct.pack("<I", len(data)))
                req.append(data)
            buf = memoryview(b"".join(req))
            while buf:   # an unbuffered pipe write may take part of the request
                buf = buf[p.stdin.write(buf):]
            out: Dict[str, Optional[np.ndarray]] = {}
            for name, _ in items:
                h, w = struct.unpack("<ii", _read_exact(p.stdout, 8))
                if h < 0:
                    out[name] = None
                    continue
                raw = _read_exact(p.stdout, h * w * 3)
                out[name] = np.frombuffer(raw, np.uint8).reshape(h, w, 3)
            self.free.put(p)
            return out
        except Exception:
            # a worker that failed mid-chunk (died, or its pipe is out of step) is replaced, so
            # the pool never shrinks; the caller decodes this chunk in-process
            p.kill()
            try:
                p.wait(timeout=5)   # reap it
            except subprocess.TimeoutExpired:
                pass
            try:
                p = self._spawn()
            except Exception:       # the slot comes back anyway (a dead worker fails fast and
                pass                # is replaced again), so free.get() never waits on a lost slot
            self.free.put(p)
            raise

    def close(self) -> None:
        with self._lock:
            if self.closed:
                return
            self.closed = True
        for p in self.procs:
            try:
                p.stdin.close()
            except OSError:
                pass
        for p in self.procs:
            try:
                p.wait(timeout=5)
            except subprocess.TimeoutExpired:
                p.kill()


if __name__ == "__main__":
    _serve()
