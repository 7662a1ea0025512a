#!/usr/bin/env python3
"""Time the GPU JPEG path (csrc/kernels/jpeg_decode.hip) on one store-image window: host
prepare (parse + un-stuff, native) and the device decode + resize of --n synthetic bench JPEGs
(service_bench.make_jpegs: 300 x 169-300, ~15 KB), against the CPU decode workers.

  python tools/jpeg_bench.py [--n 256] [--hw 224] [--iters 10]
  rocprofv3 --kernel-trace --stats -d gpurun_out/jpeg -- python3 tools/jpeg_bench.py
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_machine_learning_amd import _native as N  # noqa: E402
from distributed_machine_learning_amd.parallel.rank_backend import _JpegPack  # noqa: E402
from distributed_machine_learning_amd.parallel.service_bench import make_jpegs  # noqa: E402


class _Pins:
    def __init__(self, k=1):
        self.streams = [torch.cuda.Stream() for _ in range(k)]
        self.i = 0

    def jpeg_stream(self):
        self.i = (self.i + 1) % len(self.streams)
        return self.streams[self.i]

    device = torch.device("cuda")

    def remember_planes(self, pack, recs):
        pass

    def pinned(self, nbytes):
        return torch.empty(nbytes, dtype=torch.uint8).pin_memory()

    def unpin(self, buf):
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--hw", type=int, default=224)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--windows", type=int, default=4, help="windows in flight on as many side streams")
    a = ap.parse_args()
    N.ensure_device_init()
    N.check(N.lib().dml_jpeg_init(), "dml_jpeg_init")
    files = make_jpegs(a.n, seed=11)
    names, datas = [n for n, _ in files], [d for _, d in files]
    arena = torch.zeros((a.n, a.hw, a.hw, 3), dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    prep, dev = [], []
    for it in range(a.iters + 2):
        t0 = time.perf_counter()
        pack = _JpegPack(_Pins(), names, datas, (a.hw, a.hw))
        t1 = time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        pack.launch(list(range(len(pack.names))), arena, s)
        e1.record(s)
        e1.synchronize()
        if it >= 2:
            prep.append((t1 - t0) * 1e3)
            dev.append(e0.elapsed_time(e1))
        pack.release()
    prep.sort()
    dev.sort()
    print(f"window of {a.n} JPEGs -> {a.hw}x{a.hw}: host prepare {prep[len(prep) // 2]:.2f} ms, "
          f"device (H2D + huffman + idct + rgb/resize) {dev[len(dev) // 2]:.2f} ms "
          f"= {a.n / (dev[len(dev) // 2] / 1e3):.0f} images/s on an idle GPU", flush=True)
    # several windows in flight, each on its own side stream (as GpuRankBackend.jpeg_stream)
    pins = _Pins(a.windows)
    packs = [_JpegPack(pins, names, datas, (a.hw, a.hw)) for _ in range(a.windows)]
    big = torch.zeros((a.windows * a.n, a.hw, a.hw, 3), dtype=torch.uint8, device="cuda")
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k, pk in enumerate(packs):
            pk.launch(list(range(k * a.n, k * a.n + len(pk.names))), big, s)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(f"{a.windows} windows on {a.windows} side streams: {dt * 1e3:.2f} ms = "
          f"{a.windows * a.n / dt:.0f} images/s", flush=True)


if __name__ == "__main__":
    main()
