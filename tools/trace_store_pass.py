#!/usr/bin/env python3
"""Store-image pass timeline from a rocprofv3 kernel-trace CSV: over the span of the GPU JPEG
kernels (the pass), the busy union of the model kernels, of the JPEG kernels (Huffman, IDCT,
colour + resize), of both, and the idle rest; per JPEG kernel the launches and mean time.

  python tools/trace_store_pass.py gpurun_out/prof_distinct/run_kernel_trace.csv
"""
import collections
import csv
import json
import sys


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
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    jp = [r for r in rows if "jpg::" in r[2]]
    t0, t1 = jp[0][0], max(r[1] for r in jp)
    win = [r for r in rows if t0 <= r[0] <= t1]
    model = [(s, e) for s, e, n in win if "jpg::" not in n and "rocclr" not in n and "at::" not in n]
    jpeg = [(s, e) for s, e, n in win if "jpg::" in n]
    per = collections.defaultdict(list)
    for s, e, n in jp:
        per[n.split("(")[0]].append(e - s)
    out = {"span_ms": round((t1 - t0) / 1e6, 2),
           "model_union_ms": round(union(model) / 1e6, 2), "jpeg_union_ms": round(union(jpeg) / 1e6, 2),
           "any_union_ms": round(union(model + jpeg) / 1e6, 2),
           "idle_ms": round((t1 - t0 - union(model + jpeg)) / 1e6, 2),
           "jpeg_kernels": {k: {"n": len(v), "mean_us": round(sum(v) / len(v) / 1e3, 1)} for k, v in per.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
