#!/usr/bin/env python3
"""Chained-GEMM block boundary (expand_reduce_chain.hip) vs the two tuned 1x1
launches it replaces, ResNet50 stage 3 (F = 128, C = 512), 128-image sub-batch,
cold (L2/MALL scrubbed before each launch) and warm.

  python tools/chain_bench.py --out gpurun_out/chain.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--c", type=int, default=512, choices=(512, 1024), help="512: stage 3 (28x28), 1024: stage 4 (14x14)")
    a = ap.parse_args()
    import torch

    from distributed_machine_learning_amd import ops
    from distributed_machine_learning_amd.ops import tuning

    torch.manual_seed(0)
    h = w = 28 if a.c == 512 else 14
    c, f = a.c, a.c // 4
    m = a.n * h * w
    x = torch.randn(a.n, h, w, f, device="cuda").clamp(min=0).to(torch.bfloat16)
    res = torch.randn(a.n, h, w, c, device="cuda").to(torch.bfloat16)
    w3 = (torch.randn(c, f) * (2.0 / f) ** 0.5).view(c, f, 1, 1)
    w1 = (torch.randn(f, c) * (2.0 / c) ** 0.5).view(f, c, 1, 1)
    b3, b1 = torch.randn(c) * 0.1, torch.randn(f) * 0.1
    w3p, _, _ = ops.pack_weight(w3)
    w1p, _, _ = ops.pack_weight(w1)
    w3p, w1p = w3p.cuda(), w1p.cuda()
    scrub = torch.zeros(128 << 20, device="cuda")

    def timed(fn, cold):
        fn()
        torch.cuda.synchronize()
        ms = 0.0
        for _ in range(a.iters):
            if cold:
                scrub.add_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ms += e0.elapsed_time(e1)
        return round(ms / a.iters * 1e3, 2)

    # the two launches on their tuned tiles
    d = []
    ops.conv2d_nhwc(x, w3p, b3, c, 1, 1, relu=True, residual=res, defer=d)
    y = torch.empty(a.n, h, w, c, device="cuda", dtype=torch.bfloat16)
    z = torch.empty(a.n, h, w, f, device="cuda", dtype=torch.bfloat16)
    ops.conv2d_nhwc(y, w1p, b1, f, 1, 1, relu=True, defer=d)
    tab = tuning.autotune(d, persist=False)
    cfg_e, cfg_r = tab[tuning.shape_key(d[0])], tab[tuning.shape_key(d[1])]

    def two():
        ops.conv2d_nhwc(x, w3p, b3, c, 1, 1, relu=True, residual=res, out=y, cfg=cfg_e)
        ops.conv2d_nhwc(y, w1p, b1, f, 1, 1, relu=True, out=z, cfg=cfg_r)

    def fused():
        return ops.expand_reduce(x.view(m, f), w3p, b3, res.view(m, c), w1p, b1)

    y2, z2 = fused()
    two()
    torch.cuda.synchronize()
    err_y = ((y2.float() - y.view(m, c).float()).abs().max() / y.float().abs().max()).item()
    err_z = ((z2.float() - z.view(m, f).float()).abs().max() / z.float().abs().max()).item()
    rec = {"m": m, "C": c, "F": f, "waves": os.environ.get("DML_CHAIN_WAVES", "4"), "cfgs": [cfg_e, cfg_r],
           "two_launches_cold_us": timed(two, True), "two_launches_warm_us": timed(two, False),
           "fused_cold_us": timed(fused, True), "fused_warm_us": timed(fused, False),
           "hbm_min_mb_fused": round(m * (f + c + c + f) * 2 / 1e6, 1),
           "rel_err_y": round(err_y, 5), "rel_err_z": round(err_z, 5)}
    # in-kernel phase stamps (s_memtime, wave 0 of each workgroup; a separate diagnostic launch)
    import ctypes as C

    from distributed_machine_learning_amd import _native as N

    px = 32 if c == 512 else 16
    bm = px * (8 if os.environ.get("DML_CHAIN_WAVES") == "8" else 4)
    nblk = (m + bm - 1) // bm
    st = torch.zeros(nblk * 40, dtype=torch.int64, device="cuda")
    b3d, b1d = b3.cuda().float(), b1.cuda().float()
    ea = N.ExpandReduceArgs(x.data_ptr(), w3p.data_ptr(), b3d.data_ptr(), res.data_ptr(), y2.data_ptr(),
                            w1p.data_ptr(), b1d.data_ptr(), z2.data_ptr(), m, f, w3p.shape[1], c, c, w1p.shape[1],
                            f, c, f, 0, 0, 0, st.data_ptr())
    if N.lib().dml_chain_supported(C.byref(ea)):
        for _ in range(3):
            N.check(N.lib().dml_expand_reduce(C.byref(ea), N.stream_ptr()), "chain stamps")
        torch.cuda.synchronize()
        t = st.view(nblk, 40).cpu().double()
        med = lambda v: round(float(v.median()), 1)  # noqa: E731
        ph = {"prologue": med(t[:, 1] - t[:, 0])}
        nch = c // 64  # stamps cover the first 8 chunks
        for k in range(min(nch, 8)):
            base = 2 + 4 * k
            prev = t[:, 1] if k == 0 else t[:, base - 1]
            ph[f"c{k}_gemm1"] = med(t[:, base] - prev)
            ph[f"c{k}_rwait"] = med(t[:, base + 1] - t[:, base])
            ph[f"c{k}_epi"] = med(t[:, base + 2] - t[:, base + 1])
            ph[f"c{k}_gemm2"] = med(t[:, base + 3] - t[:, base + 2])
        ph["z_out"] = med(t[:, 34] - t[:, 2 + 4 * min(nch, 8) - 1])
        ph["wg_total"] = med(t[:, 34] - t[:, 0])
        rec["stamps_cycles_median"] = ph
    print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main()
