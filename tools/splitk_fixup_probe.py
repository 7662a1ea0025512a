"""Time the in-kernel split-K variant (DmlConvArgs.fixup) against the plain
kernel on the K-heavy / under-filled ResNet50 and InceptionV3 shapes.

python tools/splitk_fixup_probe.py [--batch 128] [--iters 20]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_machine_learning_amd import _native as N, ops  # noqa: E402
from distributed_machine_learning_amd.ops import tuning  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--out", default="")
a_ = ap.parse_args()
L = N.lib()
N.ensure_device_init()
SHAPES = [  # name, h, w, cin, cout, kh, kw, pad (stride 1), batch multiplier
    ("r50 stage4 reduce K1024", 14, 14, 1024, 256, 1, 1, 0, 1),
    ("r50 stage5 reduce K2048", 7, 7, 2048, 512, 1, 1, 0, 1),
    ("r50 stage5 3x3 K4608", 7, 7, 512, 512, 3, 3, 1, 1),
    ("r50 stage4 3x3 K2304", 14, 14, 256, 256, 3, 3, 1, 1),
    ("inc 8x8 3x3 448->384", 8, 8, 448, 384, 3, 3, 1, 0.5),
    ("inc 17x17 1x7 160->160", 17, 17, 160, 160, 1, 7, 0, 0.5),
]
rows = []
for name, h, w, cin, cout, kh, kw, pad, bm in SHAPES:
    B = int(a_.batch * bm)
    ph, pw = (kh // 2, kw // 2) if pad else (0, 0 if kw == 1 else kw // 2)
    if kh == 1 and kw == 7:
        ph, pw = 0, 3
    x = torch.randn(B, h, w, cin, device="cuda").to(torch.bfloat16)
    wp, K, Kp = ops.pack_weight(torch.randn(cout, cin, kh, kw) * 0.02)
    wp = wp.cuda()
    bias = torch.zeros(256 * ((cout + 255) // 256), device="cuda")
    ho, wo = h + 2 * ph - kh + 1, w + 2 * pw - kw + 1
    y = torch.empty(B, ho, wo, cout, device="cuda", dtype=torch.bfloat16)
    a = N.ConvArgs(x.data_ptr(), wp.data_ptr(), bias.data_ptr(), None, y.data_ptr(), B, h, w, cin, cin, kh, kw,
                   1, 1, ph, pw, ho, wo, cout, K, Kp, cout, 0, 1, 0, 1, 1)
    res = {"shape": name, "M": B * ho * wo, "N": cout, "K": K, "us": {}}
    for cfg in (11, 14, 15, 26, 28, 30, 32):
        for ks in (1, 2, 3, 4):
            b = N.ConvArgs.from_buffer_copy(a)
            keep = None
            if ks > 1:
                keep = tuning.fixup_buffers(b, cfg, ks)
                b.ksplit, b.fixup, b.ws, b.tickets = ks, 1, keep[0].data_ptr(), keep[1].data_ptr()
            try:
                t = tuning.time_cfg(b, cfg, iters=a_.iters)
            except N.NativeError:
                continue
            res["us"][f"{cfg}/{ks}"] = round(t * 1e3, 1)
    best1 = min((v, k) for k, v in res["us"].items() if k.endswith("/1"))
    best = min((v, k) for k, v in res["us"].items())
    res["best_plain"], res["best"] = best1, best
    rows.append(res)
    print(f"{name:26s} M={res['M']:6d} N={cout:4d} K={K:5d}  plain {best1[1]} {best1[0]} us  best {best[1]} {best[0]} us",
          flush=True)
if a_.out:
    json.dump(rows, open(a_.out, "w"), indent=1)
