"""Microbenchmark of the conv kernel configs on the real layer shapes.

python tools/conv_bench.py [--model ResNet50] [--batch 256] [--cfgs 0,10,11] [--out file.json]
Prints per-shape time and TFLOP/s for each cfg; one process, interleaved rounds.
"""
import argparse, ctypes as C, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_machine_learning_amd import _native as N, ops
from distributed_machine_learning_amd.models import build_graph
from distributed_machine_learning_amd.models.graph import Conv

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="ResNet50"); ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--cfgs", default="10,11,12,13,14,15,16,17"); ap.add_argument("--out", default="")
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--only", default="", help="comma list of layer-name substrings to keep")
ap.add_argument("--flush", action="store_true",
                help="cold caches: overwrite a 512 MiB buffer before each timed launch (L2 + MALL evicted)")
args = ap.parse_args()
g = build_graph(args.model); B = args.batch
L = N.lib(); N.ensure_device_init()
cfgs = [int(c) for c in args.cfgs.split(",")]
def r(x, m): return (x + m - 1) // m * m
shapes = {}
for n in g.conv_nodes():
    h, w, c = g.shape(n.inp); ho, wo, _ = g.shape(n.out)
    key = (h, w, r(n.cin, 8), n.cout, n.kh, n.kw, n.sh, n.ph, n.pw, bool(n.residual))
    shapes.setdefault(key, []).append(n.name)
res = []
s = torch.cuda.current_stream()
scrub = torch.zeros(128 << 20, device="cuda") if args.flush else None  # 512 MiB
for key, names in shapes.items():
    if args.only and not any(o in names[0] for o in args.only.split(",")):
        continue
    h, w, cin, cout, kh, kw, st, ph, pw, hasres = key
    ho = (h + 2 * ph - kh) // st + 1; wo = (w + 2 * pw - kw) // st + 1
    K = kh * kw * cin; Kp = r(K, 64)
    x = torch.randn(B, h, w, cin, device="cuda").to(torch.bfloat16)
    w_oihw = torch.randn(cout, cin, kh, kw) * (2.0 / K) ** 0.5
    wt = ops.pack_weight(w_oihw)[0].cuda()
    bias = torch.zeros(r(cout, 256), device="cuda")
    y = torch.empty(B, ho, wo, cout, device="cuda", dtype=torch.bfloat16)
    rs = torch.randn(B, ho, wo, cout, device="cuda").to(torch.bfloat16) if hasres else None
    a = N.ConvArgs(x.data_ptr(), wt.data_ptr(), bias.data_ptr(), rs.data_ptr() if rs is not None else None,
                   y.data_ptr(), B, h, w, cin, cin, kh, kw, st, st, ph, pw, ho, wo, cout, K, Kp, cout,
                   cout if hasres else 0, 1, 0)
    flops = 2.0 * B * ho * wo * cout * kh * kw * cin
    nbytes = 2.0 * (B * h * w * cin + B * ho * wo * cout * (2 if hasres else 1))
    row = {"layers": names, "M": B * ho * wo, "N": cout, "K": K, "kh": kh, "kw": kw, "stride": st,
           "gflop": flops / 1e9, "mb": nbytes / 1e6, "ms": {}}
    ref = None
    variants = list(cfgs)
    for cfg in variants:
        aa = a
        kc = cfg
        try:
            N.check(L.dml_conv(C.byref(aa), cfg, N.stream_ptr()), "conv")
            torch.cuda.synchronize()
            out = y.float()
            if ref is None: ref = out
            err = ((out - ref).abs().max() / (ref.abs().max() + 1e-6)).item()
            if args.flush:
                ms = 0.0
                for _ in range(args.iters):
                    scrub.add_(1.0)
                    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
                    e0.record()
                    L.dml_conv(C.byref(aa), cfg, N.stream_ptr())
                    e1.record(); torch.cuda.synchronize()
                    ms += e0.elapsed_time(e1) / args.iters
            else:
                e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
                e0.record()
                for _ in range(args.iters):
                    L.dml_conv(C.byref(aa), cfg, N.stream_ptr())
                e1.record(); torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.iters
            row["ms"][kc] = round(ms, 4)
            row.setdefault("err", {})[kc] = round(err, 4)
        except Exception as ex:
            row["ms"][kc] = None
            print("cfg", cfg, "failed", ex)
    best = min((v, k) for k, v in row["ms"].items() if v)
    row["best"] = best[1]
    row["best_tflops"] = round(flops / best[0] / 1e9, 1)
    res.append(row)
    print(f"{names[0]:22s} x{len(names)} M={row['M']:8d} N={cout:5d} K={K:5d} " +
          " ".join(f"{c}:{row['ms'][c]}" for c in row["ms"]) + f" best={best[1]} {row['best_tflops']}TF err={row.get('err')}",
          flush=True)
tot = {c: sum((row["ms"].get(c) or 1e9) * len(row["layers"]) for row in res) for c in cfgs}
best_tot = sum(min(v for v in row["ms"].values() if v) * len(row["layers"]) for row in res)
print("total per cfg (ms):", {c: round(v, 3) for c, v in tot.items()}, "best-per-shape total:", round(best_tot, 3))
if args.out:
    json.dump({"model": args.model, "batch": B, "rows": res, "totals": tot, "best_total": best_tot}, open(args.out, "w"), indent=1)
