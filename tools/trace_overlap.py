"""Concurrency profile of a rocprofv3 kernel trace (CSV) over the last N forwards:
time with 0 / 1 / 2 / 3+ kernels in flight, and per kernel family the summed
duration and the part of it that ran alone (no other kernel in flight) — the
time a kernel's tail or a serial chain leaves the rest of the chip idle.

python tools/trace_overlap.py gpurun_out/prof/run_kernel_trace.csv [--marker stem_kernel] [--last 12]
"""
import argparse
import csv
import re
from collections import defaultdict


def family(name: str) -> str:
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    return n[:90]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="stem_kernel")
    ap.add_argument("--last", type=int, default=12)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    marks = [e for e in ev if a.marker in e[2]]
    t0 = marks[-min(a.last, len(marks))][0]
    ev = [e for e in ev if e[0] >= t0]
    t1 = max(e[1] for e in ev)
    # sweep over start/end points
    pts = sorted({t for s, e, _ in ev for t in (s, e)})
    conc = defaultdict(int)  # number in flight -> ns
    alone = defaultdict(int)
    total = defaultdict(int)
    calls = defaultdict(int)
    for s, e, n in ev:
        total[family(n)] += e - s
        calls[family(n)] += 1
    active = []
    j = 0
    for p0, p1 in zip(pts, pts[1:]):
        while j < len(ev) and ev[j][0] <= p0:
            active.append(ev[j])
            j += 1
        active = [x for x in active if x[1] > p0]
        k = len(active)
        conc[min(k, 3)] += p1 - p0
        if k == 1:
            alone[family(active[0][2])] += p1 - p0
    win = t1 - t0
    print(f"{len(ev)} kernels over {win / 1e3:.1f} us ({len(marks)} markers, last {a.last})")
    for k in range(4):
        print(f"  {k}{'+' if k == 3 else ' '} in flight: {conc[k] / 1e3:9.1f} us  {100 * conc[k] / win:5.1f} %")
    print(f"{'kernel':90s} {'calls':>6s} {'sum us':>9s} {'alone us':>9s}")
    for f in sorted(total, key=lambda f: -total[f])[:a.top]:
        print(f"{f:90s} {calls[f]:6d} {total[f] / 1e3:9.1f} {alone[f] / 1e3:9.1f}")


if __name__ == "__main__":
    main()
