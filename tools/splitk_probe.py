"""Probe: does split-K help the small-M / long-K ResNet50 layers?

Times the v2 conv kernel on a layer shape with ksplit = 1 (bf16 out, ReLU) and
ksplit = 2, 4 (fp32 partial slices, no ReLU) for a few tile configs. Prints a
JSON line per shape: {cfg: {ksplit: ms}}. The reduce of the slices is not
included (it would cost one extra ~6-25 MB streaming pass).

  python tools/splitk_probe.py [--batch 128]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_machine_learning_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
B = args.batch
# (name, H, W, Cin, Cout, k, stride, pad)
SHAPES = [("conv5_3x3", 7, 7, 512, 512, 3, 1, 1), ("conv5_reduce", 7, 7, 2048, 512, 1, 1, 0),
          ("conv4_3x3", 14, 14, 256, 256, 3, 1, 1), ("conv4_reduce", 14, 14, 1024, 256, 1, 1, 0)]
CFGS = [11, 14, 22, 26, 30, 31]


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(args.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / args.iters


for name, h, w, cin, cout, k, st, pad in SHAPES:
    x = torch.randn(B, h, w, cin, device="cuda").to(torch.bfloat16)
    wt = ops.pack_weight(torch.randn(cout, cin, k, k) * (2.0 / (cin * k * k)) ** 0.5)[0].cuda()
    b = torch.zeros(cout, device="cuda")
    res = {}
    for cfg in CFGS:
        r = {}
        for ks in (1, 2, 4):
            try:
                if ks == 1:
                    f = lambda: ops.conv2d_nhwc(x, wt, b, cout, k, k, (st, st), (pad, pad), relu=True, cfg=cfg)
                else:
                    f = lambda: ops.conv2d_nhwc(x, wt, b, cout, k, k, (st, st), (pad, pad), out_f32=True, cfg=cfg,
                                                ksplit=ks)
                r[ks] = round(timeit(f), 4)
            except Exception as e:  # config cannot run this shape
                r[ks] = str(e)[:40]
        res[cfg] = r
    print(json.dumps({"shape": name, "batch": B, "ms": res}), flush=True)
