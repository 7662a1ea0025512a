"""Roofline table of the stride-1 3x3 convs: direct implicit-GEMM tiles vs the Winograd
kernels (tools/wino_bench.py output), per layer shape and summed per forward.

python tools/wino_roofline.py profiles/r4_wino/wino_bench_cfg80-83.json > profiles/r4_wino/conv3x3_roofline.csv

Bounds: MFMA = direct MACs at the dense bf16 peak (2.5 PFLOP/s; Winograd: its 16/36 of
them), HBM = input + output bytes at 8 TB/s (Winograd's transformed operands stay on chip)."""
import json
import sys

PEAK, HBM = 2.5e15, 8e12
# layers of each shape per forward sub-batch (ResNet50 per 128 images after the stride
# pushdown, InceptionV3 per 64 images)
COUNT = {"r50_s2": 2, "r50_s3": 3, "r50_s4": 5, "r50_s5": 3, "inc_c5": 1, "inc_35_64_96": 3,
         "inc_35_96_96": 3, "inc_8_448_384": 2}
SHAPES = {"r50_s2": (128, 56, 56, 64, 64, 1), "r50_s3": (128, 28, 28, 128, 128, 1),
          "r50_s4": (128, 14, 14, 256, 256, 1), "r50_s5": (128, 7, 7, 512, 512, 1),
          "inc_c5": (64, 73, 73, 80, 192, 0), "inc_35_64_96": (64, 35, 35, 64, 96, 1),
          "inc_35_96_96": (64, 35, 35, 96, 96, 1), "inc_8_448_384": (64, 8, 8, 448, 384, 1)}


def main(path):
    rows = json.load(open(path))
    print("shape,count,gflop_direct,mfma_bound_us,wino_mfma_bound_us,hbm_bound_us,direct_best_cold_us,direct_cfg,"
          "wino_best_cold_us,wino_cfg,wino_vs_direct")
    tot = {"r50": [0, 0, 0], "inc": [0, 0, 0]}
    for r in rows:
        n, h, w, ci, co, pad = SHAPES[r["shape"]]
        ho, wo = h + 2 * pad - 2, w + 2 * pad - 2
        gf = r["gflop_direct"]
        mb = gf * 1e9 / PEAK * 1e6
        hb = (n * h * w * ci + n * ho * wo * co) * 2 / HBM * 1e6
        us = r["us"]
        d = min((v["cold"], k) for k, v in us.items() if int(k.split(":")[1]) < 80)
        wn = min(((v["cold"], k) for k, v in us.items() if int(k.split(":")[1]) >= 80), default=(float("nan"), "-"))
        c = COUNT[r["shape"]]
        print(f"{r['shape']},{c},{gf:.2f},{mb:.1f},{mb * 16 / 36:.1f},{hb:.1f},{d[0]:.1f},{d[1]},{wn[0]:.1f},{wn[1]},"
              f"{wn[0] / d[0]:.2f}")
        m = tot["r50" if r["shape"].startswith("r50") else "inc"]
        m[0] += c * d[0]
        m[1] += c * min(d[0], wn[0])
        m[2] += c * max(mb, hb)
    for k, (d, b, rl) in tot.items():
        print(f"# {k}: 3x3/1 total {d:.0f} us direct, {b:.0f} us best-of-both, roofline {rl:.0f} us "
              f"({'per 128 images' if k == 'r50' else 'per 64 images'})")


if __name__ == "__main__":
    main(sys.argv[1])
