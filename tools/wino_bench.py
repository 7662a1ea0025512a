"""Winograd F(2x2, 3x3) kernel (cfg 80) vs the implicit-GEMM tiles on the stride-1 3x3
shapes of ResNet50 (sub-batch 128) and InceptionV3 (sub-batch 64), warm and cold.

python tools/wino_bench.py [--cfgs 80,11,15,30,32] [--iters 20] [--out file.json] [--lib path.so,...]
--lib: extra library builds (kernel variants) timed on the same shapes (DML_LIB per process is not
possible in one process, so each variant library is loaded under its own ctypes handle).
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_machine_learning_amd import _native as N, ops  # noqa: E402

SHAPES = [  # name, batch, h, w, cin, cout, pad
    ("r50_s2", 128, 56, 56, 64, 64, 1), ("r50_s3", 128, 28, 28, 128, 128, 1),
    ("r50_s4", 128, 14, 14, 256, 256, 1), ("r50_s5", 128, 7, 7, 512, 512, 1),
    ("inc_c5", 64, 73, 73, 80, 192, 0), ("inc_35_64_96", 64, 35, 35, 64, 96, 1),
    ("inc_35_96_96", 64, 35, 35, 96, 96, 1), ("inc_8_448_384", 64, 8, 8, 448, 384, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="80,11,15,30,32,12,14")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--out", default="")
    ap.add_argument("--lib", default="", help="comma list of variant libraries (their cfg 80 is timed)")
    a = ap.parse_args()
    libs = [("main", N.lib())]
    N.ensure_device_init()
    for p in [x for x in a.lib.split(",") if x]:
        L2 = C.CDLL(p)
        L2.dml_conv.argtypes = [C.POINTER(N.ConvArgs), C.c_int, C.c_void_p]
        L2.dml_conv_v2_init()
        libs.append((os.path.basename(p), L2))
    scrub = torch.zeros(128 << 20, device="cuda")
    s = N.stream_ptr()
    rows = []
    for name, B, h, w, cin, cout, pad in SHAPES:
        if a.only and a.only not in name:
            continue
        torch.manual_seed(0)
        ho, wo = h + 2 * pad - 2, w + 2 * pad - 2
        x = torch.randn(B, h, w, cin, device="cuda").to(torch.bfloat16)
        wt = torch.randn(cout, cin, 3, 3) * (2.0 / (9 * cin)) ** 0.5
        wp, K, kp = ops.pack_weight(wt)
        wp, wu = wp.cuda(), ops.pack_wino_weight(wt).cuda()
        bias = torch.zeros(wp.shape[0], device="cuda")
        y = torch.empty(B, ho, wo, cout, device="cuda", dtype=torch.bfloat16)
        args = N.ConvArgs(x.data_ptr(), wp.data_ptr(), bias.data_ptr(), None, y.data_ptr(), B, h, w, cin, cin, 3, 3,
                          1, 1, pad, pad, ho, wo, cout, K, kp, cout, 0, 1, 0, 1, 1)
        args.wu = wu.data_ptr()
        gflop = 2.0 * B * ho * wo * cout * 9 * cin / 1e9
        row = {"shape": name, "gflop_direct": gflop, "us": {}}
        todo = [(f"{ln}:{c}", L, c) for c in [int(c) for c in a.cfgs.split(",")] for ln, L in libs
                if ln == "main" or c == 80]
        for label, L, cfg in todo:
            def run():
                rc = L.dml_conv(C.byref(args), cfg, s)
                if rc != 0:
                    raise RuntimeError(f"{label} rc {rc}")
            try:
                run()
                torch.cuda.synchronize()
            except RuntimeError:
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            e1.synchronize()
            warm = e0.elapsed_time(e1) / a.iters * 1e3
            cold = 0.0
            for _ in range(a.iters):
                scrub.add_(1.0)
                e0.record()
                run()
                e1.record()
                e1.synchronize()
                cold += e0.elapsed_time(e1)
            cold = cold / a.iters * 1e3
            row["us"][label] = {"warm": round(warm, 2), "cold": round(cold, 2),
                                "tflops_equiv_warm": round(gflop / warm * 1e-3, 1)}
        rows.append(row)
        best = min(((v["cold"], k) for k, v in row["us"].items() if not k.endswith(":80")), default=(0, "-"))
        wino = {k: v for k, v in row["us"].items() if k.endswith(":80")}
        print(f"{name:16s} direct best cold {best[0]:7.1f} us ({best[1]})  wino " +
              "  ".join(f"{k} {v['warm']:.1f}/{v['cold']:.1f}" for k, v in wino.items()), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
