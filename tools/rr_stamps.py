#!/usr/bin/env python3
"""Phase timestamps of the row-ring 3x3 kernel (csrc/kernels/conv_rowring.hip,
dml_conv_rr_stamped): per workgroup, wave 0 stamps the kernel start, then per tile the moments
before its vmcnt wait, after the tile's barrier, after its MFMAs (with the next rows' DMA and the
previous tile's stores interleaved) and after the epilogue. Prints median phase lengths over the workgroups (s_memtime ticks = shader cycles).

  python tools/rr_stamps.py [--batch 128] [--cfg 150] [--cold]
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributed_machine_learning_amd import _native as N, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--cfg", type=int, default=150)
    ap.add_argument("--cold", action="store_true")
    a = ap.parse_args()
    N.ensure_device_init()
    L, s = N.lib(), N.stream_ptr()
    f = L.dml_conv_rr_stamped
    f.restype = C.c_int
    f.argtypes = [C.POINTER(N.ConvArgs), C.c_int, C.c_void_p, C.c_void_p]
    B, h, w, cin, cout = a.batch, 56, 56, 64, 64
    x = torch.randn(B, h, w, cin, device="cuda").to(torch.bfloat16)
    wp, K, kp = ops.pack_weight(torch.randn(cout, cin, 3, 3) * 0.05)
    wp = wp.cuda()
    bias = torch.zeros(wp.shape[0], device="cuda")
    y = torch.empty(B, h, w, cout, device="cuda", dtype=torch.bfloat16)
    ar = N.ConvArgs(x.data_ptr(), wp.data_ptr(), bias.data_ptr(), None, y.data_ptr(), B, h, w, cin, cin, 3, 3,
                    1, 1, 1, 1, h, w, cout, K, kp, cout, 0, 1, 0, 1, 1)
    strips = {150: 2, 151: 1, 152: 4}[a.cfg]
    grid = B * strips
    st = torch.zeros(grid * 2 * 64, dtype=torch.int64, device="cuda")
    scrub = torch.zeros(128 << 20, device="cuda") if a.cold else None
    for it in range(4):
        if scrub is not None:
            scrub.add_(1.0)
        st.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        N.check(f(C.byref(ar), a.cfg, C.c_void_p(st.data_ptr()), s), "rr stamped")
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
    t = st.view(grid, 2, 64).cpu().numpy().astype(np.int64)
    ntile = (h + 3) // 4
    per = [ntile * (i + 1) // strips - ntile * i // strips for i in range(strips)]
    nt = min(per)
    m = t[:, 0]
    t0 = m[:, 0].min()
    print(f"cfg {a.cfg} batch {B} {'cold' if a.cold else 'warm'}: {ms * 1000:.1f} us, grid {grid}, tiles/strip {per}")
    print(f"  first MFMA-wave start after kernel's first: median {np.median(m[:, 0] - t0):.0f} max {np.max(m[:, 0] - t0):.0f} cyc")
    print(f"  prologue (start -> after A0): median {np.median(m[:, 2] - m[:, 0]):.0f} cyc")
    print(" tile | wait+barrier | MFMAs (+DMA, stores) | epilogue | to next tile")
    for k in range(nt):
        b = 1 + 4 * k
        aw = np.median(m[:, b + 1] - m[:, b])
        mf = np.median(m[:, b + 2] - m[:, b + 1])
        ep = np.median(m[:, b + 3] - m[:, b + 2])
        nx = np.median(m[:, b + 4] - m[:, b + 3]) if k + 1 < nt else float("nan")
        print(f" {k:4d} | {aw:12.0f} | {mf:20.0f} | {ep:8.0f} | {nx:8.0f}")
    end = m[:, 1 + 4 * (nt - 1) + 3]
    print(f"  last MFMA stamp - first start: median {np.median(end - t0):.0f} max {np.max(end - t0):.0f} cyc")


if __name__ == "__main__":
    main()
