"""Vendor-library ceiling for the conv GEMM shapes: time torch.mm (hipBLASLt)
in bf16 on the plain GEMM of every ResNet50 / InceptionV3 conv (M = pixels,
N = Cout, K = kh*kw*Cin), i.e. without the implicit-im2col gather. Prints
per-shape TFLOP/s next to our conv kernel's time from a conv_bench JSON.

python tools/gemm_ref.py --model ResNet50 --batch 128 [--only _2_conv]
"""
import argparse, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_machine_learning_amd.models import build_graph

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="ResNet50"); ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--only", default=""); ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--out", default="")
a = ap.parse_args()
g = build_graph(a.model)
seen, rows = set(), []
for n in g.conv_nodes():
    if a.only and not any(o in n.name for o in a.only.split(",")):
        continue
    ho, wo, _ = g.shape(n.out)
    M, N, K = a.batch * ho * wo, n.cout, n.kh * n.kw * n.cin
    if (M, N, K) in seen:
        continue
    seen.add((M, N, K))
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.mm(x, w)
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(a.iters):
        torch.mm(x, w)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    tf = 2.0 * M * N * K / ms / 1e9
    rows.append({"layer": n.name, "M": M, "N": N, "K": K, "ms": round(ms, 4), "tflops": round(tf, 1)})
    print(f"{n.name:24s} M={M:7d} N={N:5d} K={K:5d} {ms*1e3:8.1f}us {tf:7.1f}TF", flush=True)
if a.out:
    json.dump(rows, open(a.out, "w"), indent=1)
