#!/usr/bin/env python3
"""Fused whole-bottleneck kernel vs the same ResNet50 block as three tuned
launches (reduce, 3x3, expand + shortcut), per 128-image sub-batch.

Timing: every launch cold (a 512 MiB buffer overwritten first, as inside a
forward: ops/tuning.py) and warm (back to back); the unfused side uses the best
tile config per conv from a cold sweep over every candidate (= the tuner).

  python tools/block_bench.py [--n 128] [--hw 56] [--f 64] [--iters 10]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--hw", type=int, default=56)
    ap.add_argument("--f", type=int, default=64)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    from distributed_machine_learning_amd import _native as N
    from distributed_machine_learning_amd import ops
    from distributed_machine_learning_amd.ops import tuning

    dev = "cuda"
    f, c, n, hw = a.f, 4 * a.f, a.n, a.hw
    g = torch.Generator().manual_seed(0)
    w1 = torch.randn(f, c, 1, 1, generator=g) * (2.0 / c) ** 0.5
    w2 = torch.randn(f, f, 3, 3, generator=g) * (2.0 / (9 * f)) ** 0.5
    w3 = torch.randn(c, f, 1, 1, generator=g) * (0.5 / f) ** 0.5
    b1, b2, b3 = (torch.randn(k, generator=g) * 0.1 for k in (f, f, c))
    x = torch.randn(n, hw, hw, c, generator=g).to(torch.bfloat16).to(dev)
    w1p, w2p, w3p = (ops.pack_weight(t)[0].to(dev) for t in (w1, w2, w3))
    scrub = torch.zeros(128 << 20, device=dev)

    def timeit(fn, cold):
        fn()
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.iters):
            if cold:
                scrub.add_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        ms.sort()
        return ms[len(ms) // 2] * 1e3  # median, us

    y = torch.empty_like(x)
    fused = {"cold_us": timeit(lambda: ops.block_fused(x, w1p, b1, w2p, b2, w3p, b3, out=y), True),
             "warm_us": timeit(lambda: ops.block_fused(x, w1p, b1, w2p, b2, w3p, b3, out=y), False),
             "phased_cold_us": timeit(lambda: ops.block_fused(x, w1p, b1, w2p, b2, w3p, b3, out=y, kernel=1), True),
             "phased_warm_us": timeit(lambda: ops.block_fused(x, w1p, b1, w2p, b2, w3p, b3, out=y, kernel=1), False)}
    # unfused: each conv on its cold-tuned best cfg
    t1 = torch.empty(n, hw, hw, f, dtype=torch.bfloat16, device=dev)
    t2 = torch.empty_like(t1)
    y3 = torch.empty_like(x)
    convs = [
        ("reduce", [], dict(x=x, w=w1p, b=b1, cout=f, k=1, pad=0, res=None, out=t1)),
        ("3x3", [], dict(x=t1, w=w2p, b=b2, cout=f, k=3, pad=1, res=None, out=t2)),
        ("expand", [], dict(x=t2, w=w3p, b=b3, cout=c, k=1, pad=0, res=x, out=y3)),
    ]
    unf = {}
    for name, d, kw in convs:
        ops.conv2d_nhwc(kw["x"], kw["w"], kw["b"], kw["cout"], kw["k"], kw["k"], pad=(kw["pad"], kw["pad"]),
                        relu=True, residual=kw["res"], out=kw["out"], defer=d)
        args = d[0]
        best = min((tuning.time_cfg(args, cfg), cfg) for cfg in tuning.valid_cfgs(args))
        L, s = N.lib(), N.stream_ptr()
        fn = (lambda args=args, cfg=best[1]: L.dml_conv(C.byref(args), cfg, s))
        unf[name] = {"cfg": best[1], "cold_us": timeit(fn, True), "warm_us": timeit(fn, False)}
    # phase stamps of one cold fused launch (diagnostic: wave 0 of each workgroup)
    nblk = n * ((hw + 13) // 14) ** 2
    st = torch.zeros(nblk * 8, dtype=torch.int64, device=dev)
    scrub.add_(1.0)
    ops.block_fused(x, w1p, b1, w2p, b2, w3p, b3, out=y, stamps=st, kernel=1)
    torch.cuda.synchronize()
    s = st.view(nblk, 4, 2).cpu().double()
    rt = s[:, :, 0]  # 100 MHz real-time ticks
    t0 = rt[:, 0].min()
    ph = {f"phase{i + 1}_us_median": round(float((rt[:, i + 1] - rt[:, i]).median()) / 100.0, 2) for i in range(3)}
    ph["wg_us_median"] = round(float((rt[:, 3] - rt[:, 0]).median()) / 100.0, 2)
    ph["kernel_span_us"] = round(float(rt[:, 3].max() - t0) / 100.0, 2)
    ph["clock_ghz"] = round(float(((s[:, 3, 1] - s[:, 0, 1]) / (rt[:, 3] - rt[:, 0])).median()) / 10.0, 3)
    fused["stamps"] = ph
    ops.block_fused(x, w1p, b1, w2p, b2, w3p, b3, out=y)  # the default (checked below)
    torch.cuda.synchronize()
    d = (y.float() - y3.float()).abs().max().item()
    res = {"n": n, "hw": hw, "F": f, "C": c, "fused": fused, "unfused": unf,
           "unfused_cold_sum_us": round(sum(v["cold_us"] for v in unf.values()), 2),
           "unfused_warm_sum_us": round(sum(v["warm_us"] for v in unf.values()), 2),
           "max_abs_diff_vs_unfused": d,
           "hbm_min_mb": round((2 * n * hw * hw * c * 2) / 1e6, 1)}
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as fo:
            json.dump(res, fo, indent=1)


if __name__ == "__main__":
    main()
