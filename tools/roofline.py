"""Per-layer roofline table of one engine forward (per-op times from
``bench.py --op-times``): FLOPs and a minimum-bytes estimate per op from the
engine's optimised graph (models/optimize.py), achieved TFLOP/s and GB/s, and
the fraction of the MI355X dense bf16 peak (2.5 PFLOP/s) and of the measured
HBM copy bandwidth (6.3 TB/s, MI355X_MICROARCH.md). The bound column is the
larger of the two fractions' time lower bounds (compute vs memory).

python tools/roofline.py profiles/r2_v1/op_times.json --model ResNet50 --out profiles/r2_v1/roofline_resnet50.csv
"""
import argparse
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_machine_learning_amd.models import build_model  # noqa: E402
from distributed_machine_learning_amd.models.graph import Conv, Dense, FusedConv, GlobalAvgPool, Pool  # noqa: E402
from distributed_machine_learning_amd.models.optimize import optimize  # noqa: E402

PEAK_TF, HBM_TBS = 2500.0, 6.3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("op_times")
    ap.add_argument("--model", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    d = json.load(open(a.op_times))
    model = a.model or d["model"]
    B = int(d["batch"])
    g0, w = build_model(model, seed=0, calibrate=False)
    g = optimize(g0, stride_push=True, weights=w)
    by_name = {}
    for n in g.nodes:
        by_name[n.name] = n
        for m in getattr(n, "members", []) or []:
            by_name[m.name] = m

    def conv_cost(n):
        ho, wo, _ = g.shape(n.out)
        h, w_, _ = g.shape(n.inp)
        fl = 2.0 * B * ho * wo * n.cout * n.kh * n.kw * n.cin
        by = 2.0 * (B * h * w_ * n.cin + B * ho * wo * n.cout + n.kh * n.kw * n.cin * n.cout)
        if n.residual:
            by += 2.0 * B * ho * wo * n.cout
        return fl, by

    rows = []
    readers = {}
    for n in g.nodes:
        for m in (getattr(n, "members", None) or [n]):
            for t in (getattr(m, "inp", None), getattr(m, "residual", None)):
                if t:
                    readers.setdefault(t, set()).add(n.name)
    for name, ms in d["ops"]:
        parts = [name] if name in by_name else [p for p in name.replace("|", "+").split("+") if p in by_name]
        fl = by = 0.0
        kinds = []
        for p in parts:
            n = by_name[p]
            if isinstance(n, Conv):
                f, b = conv_cost(n)
                kinds.append(f"conv{n.kh}x{n.kw}/{n.sh}")
            elif isinstance(n, FusedConv):
                f = b = 0.0
                for m in n.members:
                    f2, b2 = conv_cost(m)
                    f += f2
                    b += b2
                h, w_, _ = g.shape(n.inp)
                b -= 2.0 * B * h * w_ * n.cin * (len(n.members) - 1)  # the input is read once
                kinds.append(f"fused1x1x{len(n.members)}")
            elif isinstance(n, Dense):
                f, b = 2.0 * B * n.cin * n.cout, 2.0 * (B * n.cin + n.cin * n.cout) + 4.0 * B * n.cout
                kinds.append("dense")
            elif isinstance(n, Pool):
                h, w_, c = g.shape(n.inp)
                ho, wo, co = g.shape(n.out)
                f, b = 0.0, 2.0 * B * (h * w_ * c + ho * wo * co)
                kinds.append(f"{n.mode}pool")
            elif isinstance(n, GlobalAvgPool):
                h, w_, c = g.shape(n.inp)
                f, b = 0.0, 2.0 * B * h * w_ * c
                kinds.append("gap")
            else:
                f = b = 0.0
            fl += f
            by += b
        if len(parts) > 1:  # fused chain: an intermediate read only inside the chain never reaches HBM
            for p in parts[:-1]:
                n = by_name[p]
                if isinstance(n, (Conv, Pool)) and readers.get(n.out, set()) <= set(parts):
                    ho, wo, _ = g.shape(n.out)
                    by -= 2.0 * 2.0 * B * ho * wo * (n.cout if isinstance(n, Conv) else g.shape(n.out)[2])
        us = ms * 1e3
        tf = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        gbs = max(by, 0.0) / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        t_compute = fl / (PEAK_TF * 1e12) * 1e6
        t_mem = max(by, 0.0) / (HBM_TBS * 1e12) * 1e6
        rows.append({"op": name, "kind": "+".join(kinds) or name.split("_")[0], "us": round(us, 1),
                     "gflop": round(fl / 1e9, 3), "mbytes_min": round(max(by, 0.0) / 1e6, 2),
                     "tflops": round(tf, 1), "pct_bf16_peak": round(100 * tf / PEAK_TF, 1),
                     "gbs": round(gbs, 1), "pct_hbm": round(100 * gbs / (HBM_TBS * 1e3), 1),
                     "roofline_us": round(max(t_compute, t_mem), 1),
                     "bound": "compute" if t_compute >= t_mem else "memory",
                     "pct_of_roofline": round(100 * max(t_compute, t_mem) / us, 1) if us > 0 else 0.0})
    tot = sum(r["us"] for r in rows)
    roof = sum(r["roofline_us"] for r in rows)
    print(f"{model} sub-batch {B}: {tot:.0f} us measured, {roof:.0f} us roofline ({100 * roof / tot:.0f} %), "
          f"{sum(r['gflop'] for r in rows) / (tot * 1e-6) / 1e3:.0f} TFLOP/s average")
    for r in sorted(rows, key=lambda r: -r["us"])[:12]:
        print(f"  {r['op'][:44]:44s} {r['kind'][:20]:20s} {r['us']:7.1f} us {r['tflops']:6.0f} TF "
              f"{r['pct_bf16_peak']:5.1f} % peak {r['gbs']:6.0f} GB/s  {r['pct_of_roofline']:5.1f} % of roofline")
    if a.out:
        with open(a.out, "w", newline="") as f:
            wr = csv.DictWriter(f, fieldnames=list(rows[0]))
            wr.writeheader()
            wr.writerows(rows)


if __name__ == "__main__":
    main()
