"""A/B of a variant library build (tools/build_variant.py) against the main library on the
conv tile configs, per layer shape: outputs must be bit-identical; times warm and cold.

python tools/conv_ab.py --lib variants/libdml_x.so [--cfgs 11,14,15,24,25,30,31] [--iters 20] [--out f.json]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_machine_learning_amd import _native as N, ops  # noqa: E402

SHAPES = [  # name, batch, h, w, cin, cout, k, stride, pad
    ("r50_3x3_s2", 128, 56, 56, 64, 64, 3, 1, 1), ("r50_3x3_s3", 128, 28, 28, 128, 128, 3, 1, 1),
    ("r50_3x3_s4", 128, 14, 14, 256, 256, 3, 1, 1), ("r50_3x3_s5", 128, 7, 7, 512, 512, 3, 1, 1),
    ("r50_1x1_s2_red", 128, 56, 56, 256, 64, 1, 1, 0), ("r50_1x1_s2_exp", 128, 56, 56, 64, 256, 1, 1, 0),
    ("r50_1x1_s4_red", 128, 14, 14, 1024, 256, 1, 1, 0), ("r50_1x1_s4_exp", 128, 14, 14, 256, 1024, 1, 1, 0),
    ("inc_c5", 64, 73, 73, 80, 192, 3, 1, 0), ("inc_35_96_96", 64, 35, 35, 96, 96, 3, 1, 1),
    ("inc_17_1x1", 64, 17, 17, 768, 192, 1, 1, 0),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--cfgs", default="11,14,15,24,25,30,31")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    N.ensure_device_init()
    L2 = C.CDLL(a.lib)
    L2.dml_conv_v2_init()
    libs = [("main", N.lib()), ("variant", L2)]
    scrub = torch.zeros(128 << 20, device="cuda")
    s = N.stream_ptr()
    rows, bad = [], 0
    for name, B, h, w, cin, cout, k, st, pad in SHAPES:
        torch.manual_seed(0)
        ho, wo = (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1
        x = torch.randn(B, h, w, cin, device="cuda").to(torch.bfloat16)
        wt = torch.randn(cout, cin, k, k) * (2.0 / (k * k * cin)) ** 0.5
        wp, K, kp = ops.pack_weight(wt)
        wp = wp.cuda()
        bias = torch.zeros(wp.shape[0], device="cuda")
        row = {"shape": name, "us": {}}
        for cfg in [int(c) for c in a.cfgs.split(",")]:
            outs = {}
            for ln, L in libs:
                y = torch.empty(B, ho, wo, cout, device="cuda", dtype=torch.bfloat16)
                args = N.ConvArgs(x.data_ptr(), wp.data_ptr(), bias.data_ptr(), None, y.data_ptr(), B, h, w, cin, cin,
                                  k, k, st, st, pad, pad, ho, wo, cout, K, kp, cout, 0, 1, 0, 1, 1)

                def run():
                    rc = L.dml_conv(C.byref(args), cfg, C.c_void_p(s))
                    if rc != 0:
                        raise RuntimeError(f"{ln}:{cfg} rc {rc}")
                try:
                    run()
                    torch.cuda.synchronize()
                except RuntimeError:
                    break
                outs[ln] = y
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
                row["us"][f"{ln}:{cfg}"] = {"warm": round(warm, 2), "cold": round(cold / a.iters * 1e3, 2)}
            if len(outs) == 2 and not torch.equal(outs["main"], outs["variant"]):
                bad += 1
                row.setdefault("mismatch", []).append(cfg)
        rows.append(row)
        parts = []
        for cfg in [int(c) for c in a.cfgs.split(",")]:
            m, v = row["us"].get(f"main:{cfg}"), row["us"].get(f"variant:{cfg}")
            if m and v:
                parts.append(f"{cfg}: {m['cold']:.1f}->{v['cold']:.1f}")
        print(f"{name:16s} " + "  ".join(parts) + (f"  MISMATCH {row['mismatch']}" if "mismatch" in row else ""),
              flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
