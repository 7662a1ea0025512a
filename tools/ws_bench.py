"""The persistent weight-stationary 1x1 kernel (csrc/kernels/conv_ws.hip, cfgs 84..90)
against the v2 tiles on every 1x1 stride-1 conv shape of ResNet50 (b128) and
InceptionV3 (b64): outputs must be bit-identical to v2 tile 15 (same MFMA operand
order, same epilogue arithmetic); times cold (after a 512-MiB scrub, the tuner's
method) and warm.

python tools/ws_bench.py [--iters 20] [--out f.json]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_machine_learning_amd import _native as N, ops  # noqa: E402

SHAPES = [  # name, batch, h, w, cin, cout, residual
    ("r50_s2_64_64", 128, 56, 56, 64, 64, 0), ("r50_s2_red_256_64", 128, 56, 56, 256, 64, 0),
    ("r50_s2_exp_64_256_res", 128, 56, 56, 64, 256, 1), ("r50_s2_proj_64_256", 128, 56, 56, 64, 256, 0),
    ("r50_s3_red_512_128", 128, 28, 28, 512, 128, 0), ("r50_s3_exp_128_512_res", 128, 28, 28, 128, 512, 1),
    ("r50_s4_red_1024_256", 128, 14, 14, 1024, 256, 0), ("r50_s4_exp_256_1024_res", 128, 14, 14, 256, 1024, 1),
    ("r50_s5_exp_512_2048_res", 128, 7, 7, 512, 2048, 1),
    ("inc_35_192_64", 64, 35, 35, 192, 64, 0), ("inc_35_256_64", 64, 35, 35, 256, 64, 0),
    ("inc_35_288_64", 64, 35, 35, 288, 64, 0), ("inc_17_768_192", 64, 17, 17, 768, 192, 0),
    ("inc_8_1280_320", 64, 8, 8, 1280, 320, 0),
]
V2 = (14, 15, 32, 33, 22, 26, 12, 11, 38, 24, 27)
WS = (84, 85, 86, 87, 88, 89, 90)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="")
    ap.add_argument("--clean-scrub", action="store_true",
                    help="evict by READING 512 MiB (clean lines) instead of writing it (dirty lines whose "
                         "write-back the timed kernel pays)")
    a = ap.parse_args()
    N.ensure_device_init()
    L = N.lib()
    scrub = torch.zeros(128 << 20, device="cuda")
    sink = torch.zeros((), device="cuda")

    def evict():
        if a.clean_scrub:
            torch.sum(scrub, dim=0, out=sink)
        else:
            scrub.add_(1.0)
    s = N.stream_ptr()
    rows, bad = [], 0
    for name, B, h, w, cin, cout, res in SHAPES:
        torch.manual_seed(0)
        x = torch.randn(B, h, w, cin, device="cuda").to(torch.bfloat16)
        wt = torch.randn(cout, cin, 1, 1) * (2.0 / cin) ** 0.5
        wp, K, kp = ops.pack_weight(wt)
        wp = wp.cuda()
        bias = (torch.randn(wp.shape[0]) * 0.1).cuda()
        r = torch.randn(B, h, w, cout, device="cuda").to(torch.bfloat16) if res else None
        ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wt.cuda(), bias[:cout]).permute(0, 2, 3, 1)
        if res:
            ref = ref + r.float()
        ref = ref.relu()
        row = {"shape": name, "us": {}}
        outs = {}
        for cfg in V2 + WS:
            y = torch.empty(B, h, w, cout, device="cuda", dtype=torch.bfloat16)
            args = N.ConvArgs(x.data_ptr(), wp.data_ptr(), bias.data_ptr(), r.data_ptr() if res else None,
                              y.data_ptr(), B, h, w, cin, cin, 1, 1, 1, 1, 0, 0, h, w, cout, K, kp, cout,
                              cout if res else 0, 1, 0, 1, 1)
            if L.dml_conv(C.byref(args), cfg, C.c_void_p(s)) != 0:
                continue  # this cfg does not run this shape (channel padding / LDS size)
            torch.cuda.synchronize()
            outs[cfg] = y
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                L.dml_conv(C.byref(args), cfg, C.c_void_p(s))
            e1.record()
            e1.synchronize()
            warm = e0.elapsed_time(e1) / a.iters * 1e3
            cold = 0.0
            for _ in range(a.iters):
                evict()
                e0.record()
                L.dml_conv(C.byref(args), cfg, C.c_void_p(s))
                e1.record()
                e1.synchronize()
                cold += e0.elapsed_time(e1)
            row["us"][cfg] = {"warm": round(warm, 2), "cold": round(cold / a.iters * 1e3, 2)}
        base = outs.get(15)
        for cfg in WS:
            if cfg in outs:
                err = (outs[cfg].float() - ref).abs().max().item()
                same = base is not None and torch.equal(outs[cfg], base)
                row.setdefault("check", {})[cfg] = {"bit_equal_v2_15": same, "max_abs_err_vs_fp32": round(err, 4)}
                if not same or err > 0.05 * ref.abs().max().item() + 0.05:
                    bad += 1
        bv = min((c for c in V2 if c in row["us"]), key=lambda c: row["us"][c]["cold"], default=None)
        bw = min((c for c in WS if c in row["us"]), key=lambda c: row["us"][c]["cold"], default=None)
        row["best_v2"], row["best_ws"] = bv, bw
        msg = f"{name:26s} v2 {bv}: {row['us'][bv]['cold']:.1f}/{row['us'][bv]['warm']:.1f}" if bv else name
        if bw:
            msg += (f"  ws {bw}: {row['us'][bw]['cold']:.1f}/{row['us'][bw]['warm']:.1f}"
                    f"  x{row['us'][bv]['cold'] / row['us'][bw]['cold']:.2f} cold  "
                    + " ".join(f"{c}:{row['us'][c]['cold']:.0f}" for c in WS if c in row["us"])
                    + ("" if all(v["bit_equal_v2_15"] for v in row["check"].values()) else "  MISMATCH"))
        print(msg, flush=True)
        rows.append(row)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
