"""How far are the 1x1 conv tiles from the library GEMM on the same shapes?

For each 1x1 conv GEMM of ResNet50 / InceptionV3 at the serving batch (M = N*H*W pixels,
K = Cin, N = Cout), time (warm, back to back) torch's bf16 GEMM (hipBLASLt on ROCm:
``F.linear`` on the NHWC activation) against this repo's conv tile table (every v2 / ws /
wsp config, best of them) and print TFLOP/s of each. A probe: it decides whether 1x1
convs should go to the library GEMM (plus a fused epilogue) or stay on the hand tiles.

python tools/gemm_probe.py [--iters 20] [--out f.json]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributed_machine_learning_amd import _native as N, ops  # noqa: E402
from distributed_machine_learning_amd.ops import tuning  # noqa: E402

SHAPES = [  # name, batch, h, w, cin, cout
    ("r50_s2_red", 128, 56, 56, 256, 64), ("r50_s2_exp", 128, 56, 56, 64, 256),
    ("r50_s3_red", 128, 28, 28, 512, 128), ("r50_s3_exp", 128, 28, 28, 128, 512),
    ("r50_s4_red", 128, 14, 14, 1024, 256), ("r50_s4_exp", 128, 14, 14, 256, 1024),
    ("r50_s4_entry", 128, 14, 14, 768, 1024), ("r50_s5_red", 128, 7, 7, 2048, 512),
    ("r50_s5_exp", 128, 7, 7, 512, 2048), ("r50_s5_entry", 128, 7, 7, 1536, 2048),
    ("inc_17_1x1", 64, 17, 17, 768, 192), ("inc_8_1x1", 64, 8, 8, 2048, 448),
]


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    N.ensure_device_init()
    L, s = N.lib(), N.stream_ptr()
    rows = []
    for name, B, h, w, cin, cout in SHAPES:
        torch.manual_seed(0)
        M = B * h * w
        x = torch.randn(B, h, w, cin, device="cuda").to(torch.bfloat16)
        wt = torch.randn(cout, cin, device="cuda").to(torch.bfloat16) * 0.05
        bias = torch.randn(cout, device="cuda")
        gf = 2.0 * M * cin * cout / 1e9
        lib_us = timed(lambda: F.linear(x.view(M, cin), wt), a.iters)
        lib_epi_us = timed(lambda: torch.relu(F.linear(x.view(M, cin), wt, bias.to(torch.bfloat16))), a.iters)
        wp, K, kp = ops.pack_weight(wt.float().cpu()[:, :, None, None])
        wp = wp.cuda()
        y = torch.empty(B, h, w, cout, device="cuda", dtype=torch.bfloat16)
        ar = N.ConvArgs(x.data_ptr(), wp.data_ptr(), bias.data_ptr(), None, y.data_ptr(), B, h, w, cin, cin, 1, 1,
                        1, 1, 0, 0, h, w, cout, K, kp, cout, 0, 1, 0, 1, 1)
        best = (float("inf"), -1)
        for cfg in tuning.valid_cfgs(ar):
            if L.dml_conv(C.byref(ar), cfg, C.c_void_p(s)) != 0:
                continue
            t = timed(lambda: L.dml_conv(C.byref(ar), cfg, C.c_void_p(s)), a.iters)
            best = min(best, (t, cfg))
        r = {"shape": name, "M": M, "K": cin, "N": cout, "gflop": round(gf, 2), "lib_us": round(lib_us, 1),
             "lib_bias_relu_us": round(lib_epi_us, 1), "tile_us": round(best[0], 1), "tile_cfg": best[1],
             "lib_tflops": round(gf / lib_us * 1e3, 0), "tile_tflops": round(gf / best[0] * 1e3, 0)}
        rows.append(r)
        print(f"{name:14s} M {M:7d} K {cin:5d} N {cout:5d}  lib {lib_us:7.1f}us ({r['lib_tflops']:5.0f} TF)"
              f"  lib+bias+relu {lib_epi_us:7.1f}us  tiles {best[0]:7.1f}us cfg {best[1]:3d} ({r['tile_tflops']:5.0f} TF)",
              flush=True)
    if a.out:
        json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
