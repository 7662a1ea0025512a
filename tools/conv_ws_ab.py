"""Warp-specialised conv tiles (csrc/kernels/conv_igemm_ws.hip, cfg 100..) against the v2
tiles (conv_igemm_v2.hip) on the layer shapes of both networks: every output must be
bit-identical to the v2 reference tile (same per-element K order), times cold (L2/MALL
scrubbed before each launch, as the tuner) and warm, interleaved rounds in one process.

python tools/conv_ws_ab.py [--v2 11,14,15,...] [--ws 100,101,...] [--rounds 2] [--out f.json]
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

SHAPES = [  # name, batch, h, w, cin, cout, kh, kw, stride, ph, pw, residual
    ("r50_3x3_s2", 128, 56, 56, 64, 64, 3, 3, 1, 1, 1, 0), ("r50_3x3_s3", 128, 28, 28, 128, 128, 3, 3, 1, 1, 1, 0),
    ("r50_3x3_s4", 128, 14, 14, 256, 256, 3, 3, 1, 1, 1, 0), ("r50_3x3_s5", 128, 7, 7, 512, 512, 3, 3, 1, 1, 1, 0),
    ("r50_1x1_s2_red", 128, 56, 56, 256, 64, 1, 1, 1, 0, 0, 0), ("r50_1x1_s3_red", 128, 28, 28, 512, 128, 1, 1, 1, 0, 0, 0),
    ("r50_1x1_s4_red", 128, 14, 14, 1024, 256, 1, 1, 1, 0, 0, 0), ("r50_1x1_s5_red", 128, 7, 7, 2048, 512, 1, 1, 1, 0, 0, 0),
    ("r50_1x1_s4_exp", 128, 14, 14, 256, 1024, 1, 1, 1, 0, 0, 1), ("r50_1x1_s5_exp", 128, 7, 7, 512, 2048, 1, 1, 1, 0, 0, 1),
    ("inc_c5", 64, 73, 73, 80, 192, 3, 3, 1, 0, 0, 0), ("inc_35_64_96", 64, 35, 35, 64, 96, 3, 3, 1, 1, 1, 0),
    ("inc_35_96_96", 64, 35, 35, 96, 96, 3, 3, 1, 1, 1, 0), ("inc_17_1x7", 64, 17, 17, 160, 160, 1, 7, 1, 0, 3, 0),
    ("inc_17_7x1", 64, 17, 17, 160, 192, 7, 1, 1, 3, 0, 0), ("inc_17_1x1", 64, 17, 17, 768, 192, 1, 1, 1, 0, 0, 0),
    ("inc_8_448_384", 64, 8, 8, 448, 384, 3, 3, 1, 1, 1, 0), ("inc_8_1x3", 64, 8, 8, 384, 384, 1, 3, 1, 0, 1, 0),
    ("inc_m3_3x3s2", 64, 35, 35, 288, 384, 3, 3, 2, 0, 0, 0),
    ("inc_35_5x5", 64, 35, 35, 48, 64, 5, 5, 1, 2, 2, 0), ("inc_17_1x7_128", 64, 17, 17, 128, 128, 1, 7, 1, 0, 3, 0),
    ("inc_17_7x1_192", 64, 17, 17, 192, 192, 7, 1, 1, 3, 0, 0), ("inc_8_3x1", 64, 8, 8, 384, 384, 3, 1, 1, 1, 0, 0),
]
V2_DEFAULT = "11,12,14,15,24,25,26,28,30,31,32,33,38"
WS_DEFAULT = ",".join(str(c) for c in list(range(100, 113)) + [119] + list(range(120, 130)) + list(range(150, 153)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--v2", default=V2_DEFAULT)
    ap.add_argument("--ws", default=WS_DEFAULT)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--shapes", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    N.ensure_device_init()
    L = N.lib()
    s = N.stream_ptr()
    v2 = [int(c) for c in a.v2.split(",") if c]
    wsc = [int(c) for c in a.ws.split(",") if c]
    want = set(a.shapes.split(",")) if a.shapes else None
    rows, bad = [], 0
    for name, B, h, w, cin, cout, kh, kw, st, ph, pw, res in SHAPES:
        if want and name not in want:
            continue
        torch.manual_seed(0)
        ho, wo = (h + 2 * ph - kh) // st + 1, (w + 2 * pw - kw) // st + 1
        x = torch.randn(B, h, w, cin, device="cuda").to(torch.bfloat16)
        wt = torch.randn(cout, cin, kh, kw) * (2.0 / (kh * kw * cin)) ** 0.5
        wp, K, kp = ops.pack_weight(wt)
        wp = wp.cuda()
        bias = (torch.randn(wp.shape[0]) * 0.1).cuda()
        r = torch.randn(B, ho, wo, cout, device="cuda").to(torch.bfloat16) if res else None
        ys = {}

        def args_for(y):
            ar = N.ConvArgs(x.data_ptr(), wp.data_ptr(), bias.data_ptr(), r.data_ptr() if res else None, y.data_ptr(),
                            B, h, w, cin, cin, kh, kw, st, st, ph, pw, ho, wo, cout, K, kp, cout, cout if res else 0,
                            1, 0, 1, 1)
            return ar

        t = {c: [] for c in v2 + wsc}
        outs = {}
        for c in v2 + wsc:
            y = torch.zeros(B, ho, wo, cout, device="cuda", dtype=torch.bfloat16)
            ar = args_for(y)
            if L.dml_conv(C.byref(ar), c, C.c_void_p(s)) != 0:
                t.pop(c)
                continue
            torch.cuda.synchronize()
            outs[c] = (y, ar)
        ref_cfg = next(c for c in v2 if c in outs)
        # the patch-stationary tiles (140..) sum K chunk-major: equal to the v2 tile within bf16
        # rounding, not bit for bit; every other tile must be bit-identical
        refy = outs[ref_cfg][0].float()
        close = lambda c: ((outs[c][0].float() - refy).abs().max() / (refy.abs().max() + 1e-6)).item() < 1e-2  # noqa: E731
        mism = [c for c in outs if not (torch.equal(outs[c][0], outs[ref_cfg][0]) or (c >= 140 and close(c)))]
        if mism:
            bad += 1
        for _ in range(a.rounds):
            for c in list(t):
                ar = outs[c][1]
                t[c].append(tuning.time_cfg(ar, c, a.iters) * 1e3)
        best = {c: min(v) for c, v in t.items() if v}
        b2 = min((best[c], c) for c in v2 if c in best)
        bw = min(((best[c], c) for c in wsc if c in best), default=(float("nan"), -1))
        gf = 2.0 * B * ho * wo * cout * kh * kw * cin / 1e9
        rows.append({"shape": name, "gflop": round(gf, 2), "cold_us": {str(c): round(v, 2) for c, v in best.items()},
                     "best_v2": b2, "best_ws": bw, "mismatch": mism})
        tf = lambda us: gf / us * 1e-3 if us == us else float("nan")  # noqa: E731
        print(f"{name:16s} v2 {b2[1]:3d} {b2[0]:7.1f}us ({tf(b2[0]):5.0f} TF)  ws {bw[1]:3d} {bw[0]:7.1f}us "
              f"({tf(bw[0]):5.0f} TF)  x{b2[0] / bw[0]:.2f}" + (f"  MISMATCH {mism}" if mism else ""), flush=True)
        print("    " + " ".join(f"{c}:{best[c]:.1f}" for c in sorted(best)), flush=True)
    tuning._release_scrub()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
