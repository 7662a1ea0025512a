#!/usr/bin/env python3
"""Summary of a rocprofv3 kernel trace (CSV: ``rocprofv3 --kernel-trace --stats -d D -o run
--output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5``) of the driver's bench
command: for each model's TIMED steps (found by its stem kernel: two sub-batch forwards per
step, after the warmup's), the wall span, the GPU-busy union, the summed kernel time (sum / union =
how much the two sub-batch streams overlap), per-step busy and idle, the kernels per step, and
where the runtime's fill / copy kernels run (timed steps or elsewhere).

  python tools/driver_profile.py gpurun_out/prof_driver/run_kernel_trace.csv [--steps 20 --warmup 5]
"""
import argparse
import collections
import csv
import json


def union(iv):
    iv = sorted(iv)
    if not iv:
        return 0
    busy, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return busy + ce - cs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    ks = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Stream_Id"])))
    ks.sort()
    out = {}
    for model, stem in (("ResNet50", "stem::stem_kernel"), ("InceptionV3", "inc_stem_kernel")):
        starts = [i for i, k in enumerate(ks) if stem in k[2]]
        first = 2 * a.warmup
        last = 2 * (a.warmup + a.steps)
        if len(starts) < last:
            continue
        i0 = starts[first]
        # the timed region ends with the last kernel before the next stem launch (the verification
        # forward), i.e. the last step's softmax / top-5
        i1 = starts[last] if len(starts) > last else len(ks)
        reg = ks[i0:i1]
        t0, t1 = reg[0][0], max(k[1] for k in reg)
        iv = [(s, e) for s, e, _, _ in reg]
        busy = union(iv)
        total = sum(e - s for s, e in iv)
        # per step: from stem 2k to stem 2k+2
        steps = []
        for k in range(a.steps):
            j0, j1 = starts[first + 2 * k], starts[first + 2 * k + 2] if first + 2 * k + 2 < len(starts) else i1
            st = ks[j0:j1]
            s0, s1 = st[0][0], (ks[j1][0] if j1 < len(ks) else max(x[1] for x in st))
            steps.append(((s1 - s0) / 1e3, union([(x[0], x[1]) for x in st]) / 1e3, len(st)))
        fam = collections.Counter()
        for s, e, n, _ in reg:
            fam[n.split("(")[0].split("<")[0].replace("void ", "")] += e - s
        misc = collections.Counter(n for _, _, n, _ in reg if "rocclr" in n or "at::native" in n)
        out[model] = {
            "timed_wall_ms": round((t1 - t0) / 1e6, 3),
            "gpu_busy_union_ms": round(busy / 1e6, 3),
            "kernel_sum_ms": round(total / 1e6, 3),
            "busy_fraction": round(busy / (t1 - t0), 4),
            "stream_overlap_sum_over_union": round(total / busy, 3),
            "kernels_per_step": round(len(reg) / a.steps, 1),
            "per_step_wall_us": [round(x[0], 1) for x in steps],
            "per_step_busy_us": [round(x[1], 1) for x in steps],
            "runtime_kernels_in_timed_steps": dict(misc),
            "top_families_ms": {k: round(v / 1e6, 3) for k, v in fam.most_common(12)},
        }
    allmisc = collections.Counter(n for _, _, n, _ in ks if "rocclr" in n)
    out["runtime_kernels_whole_run"] = dict(allmisc)
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)


if __name__ == "__main__":
    main()
