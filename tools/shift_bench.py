#!/usr/bin/env python3
"""Shifted-pixel stride-1 conv (conv_shift.hip, cfg 64..) vs the best implicit-GEMM
tile (conv_igemm_v2.hip) on the stride-1 "same" conv shapes of ResNet50
(128-image sub-batch) and InceptionV3 (64-image sub-batch), cold (L2/MALL
scrubbed before each launch, the tuner's timing) and warm (back-to-back).

  python tools/shift_bench.py --out gpurun_out/shift.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    # name: n, h, w, cin, cout, kh, kw
    "r50_s2_3x3": (128, 56, 56, 64, 64, 3, 3),
    "r50_s3_3x3": (128, 28, 28, 128, 128, 3, 3),
    "r50_s4_3x3": (128, 14, 14, 256, 256, 3, 3),
    "r50_s5_3x3": (128, 7, 7, 512, 512, 3, 3),
    "inc_35_3x3_64_96": (64, 35, 35, 64, 96, 3, 3),
    "inc_35_3x3_96_96": (64, 35, 35, 96, 96, 3, 3),
    "inc_17_1x7_128": (64, 17, 17, 128, 128, 1, 7),
    "inc_17_7x1_128_192": (64, 17, 17, 128, 192, 7, 1),
    "inc_17_7x1_192": (64, 17, 17, 192, 192, 7, 1),
    "inc_8_1x3_384": (64, 8, 8, 384, 384, 1, 3),
    "inc_8_3x3_448_384": (64, 8, 8, 448, 384, 3, 3),
}
SHIFT = (64, 65, 66, 67, 68, 69)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    import torch

    from distributed_machine_learning_amd import _native as N
    from distributed_machine_learning_amd import ops
    from distributed_machine_learning_amd.ops import tuning

    res = {}
    for name, (n, h, w, cin, cout, kh, kw) in SHAPES.items():
        torch.manual_seed(0)
        x = (torch.randn(n, h, w, cin, device="cuda") * 0.5).to(torch.bfloat16)
        wt = torch.randn(cout, cin, kh, kw) * (2.0 / (cin * kh * kw)) ** 0.5
        wp, _, _ = ops.pack_weight(wt)
        wp = wp.cuda()
        b = torch.zeros(cout)
        d = []
        y = ops.conv2d_nhwc(x, wp, b, cout, kh, kw, (1, 1), (kh // 2, kw // 2), relu=True, defer=d)
        args = d[0]
        row = {"gflop": round(2.0 * n * h * w * cout * cin * kh * kw / 1e9, 3)}
        for mode in ("cold", "warm"):
            os.environ["DML_TUNE_COLD"] = "1" if mode == "cold" else "0"
            best = (1e9, -1)
            for cfg in tuning.V2_CFGS:
                try:
                    best = min(best, (tuning.time_cfg(args, cfg, a.iters), cfg))
                except N.NativeError:
                    pass
            row[f"igemm_{mode}"] = {"cfg": best[1], "us": round(best[0] * 1e3, 2)}
            sh = {}
            for cfg in SHIFT:
                try:
                    sh[cfg] = round(tuning.time_cfg(args, cfg, a.iters) * 1e3, 2)
                except N.NativeError as e:
                    sh[cfg] = str(e)[:60]
            row[f"shift_{mode}"] = sh
            ok = {c: t for c, t in sh.items() if isinstance(t, float)}
            if ok:
                c = min(ok, key=ok.get)
                row[f"speedup_{mode}"] = round(best[0] * 1e3 / ok[c], 3)
                row[f"best_shift_{mode}"] = c
        # numerics vs the implicit GEMM on the same operands
        y_ref = ops.conv2d_nhwc(x, wp, b, cout, kh, kw, (1, 1), (kh // 2, kw // 2), relu=True, cfg=11)
        errs = {}
        for cfg in SHIFT:
            try:
                yy = ops.conv2d_nhwc(x, wp, b, cout, kh, kw, (1, 1), (kh // 2, kw // 2), relu=True, cfg=cfg)
                torch.cuda.synchronize()
                errs[cfg] = round(((yy.float() - y_ref.float()).abs().max() / y_ref.float().abs().max()).item(), 5)
            except N.NativeError:
                pass
        row["rel_err_vs_igemm"] = errs
        res[name] = row
        print(name, json.dumps(row), flush=True)
        del y
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
