"""Channel-padded input probe: a conv whose Cin is not a multiple of the K tile (InceptionV3
conv2d_5: 3x3, Cin 80) has K tiles that straddle two taps (two pixel segments per 128-B
row). Time it as is and with its input stored at Cin_pad channels (zeros in the pad, weights
packed with zero rows there: ops.pack_weight(cin_eff)), on every tile config, cold (dirty
512-MiB scrub, the tuner's method) and warm; outputs compared with an fp32 reference.

python tools/cinpad_probe.py [--iters 20]
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_machine_learning_amd import _native as N, ops  # noqa: E402
from distributed_machine_learning_amd.ops.tuning import V2_CFGS  # noqa: E402

SHAPES = [  # name, batch, h, w, cin, cin_pad, cout, k, pad
    ("inc_conv2d_5", 64, 73, 73, 80, 96, 192, 3, 0),
    ("inc_conv2d_5_p128", 64, 73, 73, 80, 128, 192, 3, 0),
    ("inc_5x5_48", 64, 35, 35, 48, 64, 64, 5, 2),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    N.ensure_device_init()
    L = N.lib()
    scrub = torch.zeros(128 << 20, device="cuda")
    s = N.stream_ptr()
    for name, B, h, w, cin, cp, cout, k, pad in SHAPES:
        torch.manual_seed(0)
        ho, wo = h + 2 * pad - k + 1, w + 2 * pad - k + 1
        x = torch.randn(B, h, w, cin, device="cuda").to(torch.bfloat16)
        xp = torch.zeros(B, h, w, cp, device="cuda", dtype=torch.bfloat16)
        xp[..., :cin] = x
        wt = torch.randn(cout, cin, k, k) * (2.0 / (k * k * cin)) ** 0.5
        ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wt.cuda(), padding=pad).permute(0, 2, 3, 1)
        ref = ref.relu()
        res = {}
        for label, xx, ce in (("as_is", x, cin), (f"pad{cp}", xp, cp)):
            wp, K, kp = ops.pack_weight(wt, cin_eff=ce)
            wp = wp.cuda()
            bias = torch.zeros(wp.shape[0], device="cuda")
            best = None
            for cfg in V2_CFGS:
                y = torch.empty(B, ho, wo, cout, device="cuda", dtype=torch.bfloat16)
                args = N.ConvArgs(xx.data_ptr(), wp.data_ptr(), bias.data_ptr(), None, y.data_ptr(), B, h, w, ce, ce,
                                  k, k, 1, 1, pad, pad, ho, wo, cout, K, kp, cout, 0, 1, 0, 1, 1)
                if L.dml_conv(C.byref(args), cfg, C.c_void_p(s)) != 0:
                    continue
                torch.cuda.synchronize()
                err = (y.float() - ref).abs().max().item()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                cold = 0.0
                for _ in range(a.iters):
                    scrub.add_(1.0)
                    e0.record()
                    L.dml_conv(C.byref(args), cfg, C.c_void_p(s))
                    e1.record()
                    e1.synchronize()
                    cold += e0.elapsed_time(e1)
                cold = cold / a.iters * 1e3
                e0.record()
                for _ in range(a.iters):
                    L.dml_conv(C.byref(args), cfg, C.c_void_p(s))
                e1.record()
                e1.synchronize()
                warm = e0.elapsed_time(e1) / a.iters * 1e3
                if best is None or cold < best[1]:
                    best = (cfg, cold, warm, err)
                res.setdefault(label, []).append((cfg, round(cold, 1), round(warm, 1)))
            print(f"{name:20s} {label:7s} K {kp:5d} best cfg {best[0]}: cold {best[1]:.1f} warm {best[2]:.1f} us "
                  f"(max err {best[3]:.3f})", flush=True)
        for label, lst in res.items():
            print("   ", label, " ".join(f"{c}:{t}/{wm}" for c, t, wm in sorted(lst, key=lambda z: z[1])[:8]), flush=True)


if __name__ == "__main__":
    main()
