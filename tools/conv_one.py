#!/usr/bin/env python3
"""Launch ONE conv shape with ONE tile config back to back (for rocprofv3
counter passes: kernel-trace / --pmc runs of a single kernel).

  python tools/conv_one.py --shape r50_s4_3x3 --cfg 64 --iters 50
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shift_bench import SHAPES  # noqa: E402  (tools/ is on sys.path when run as a script)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="r50_s4_3x3", choices=sorted(SHAPES))
    ap.add_argument("--cfg", type=int, required=True)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    import torch

    from distributed_machine_learning_amd import ops

    n, h, w, cin, cout, kh, kw = SHAPES[a.shape]
    x = (torch.randn(n, h, w, cin, device="cuda") * 0.5).to(torch.bfloat16)
    wt = torch.randn(cout, cin, kh, kw) * (2.0 / (cin * kh * kw)) ** 0.5
    wp, _, _ = ops.pack_weight(wt)
    wp, b = wp.cuda(), torch.zeros(cout)
    y = ops.conv2d_nhwc(x, wp, b, cout, kh, kw, (1, 1), (kh // 2, kw // 2), relu=True, cfg=a.cfg)
    for _ in range(a.iters):
        ops.conv2d_nhwc(x, wp, b, cout, kh, kw, (1, 1), (kh // 2, kw // 2), relu=True, cfg=a.cfg, out=y)
    torch.cuda.synchronize()
    print("ok", a.shape, a.cfg, tuple(y.shape))


if __name__ == "__main__":
    main()
