"""GPU idle-gap analysis of a rocprofv3 kernel trace (CSV): union of all
kernel intervals over the last N forwards (stem kernels mark forwards); prints
total idle time and the largest gaps with the kernels around them.

python tools/trace_gaps.py gpurun_out/prof2/run_kernel_trace.csv [--marker stem_kernel] [--last 12]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--marker", default="stem_kernel")
ap.add_argument("--last", type=int, default=12)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48], r["Queue_Id"]) for r in rows)
marks = [e for e in ev if a.marker in e[2]]
t0 = marks[-min(a.last, len(marks))][0]
t1 = ev[-1][1]
busy = [(s, e) for s, e, n, q in ev if e > t0]
gaps, cur = [], busy[0][1]
for s, e in busy[1:]:
    if s > cur:
        gaps.append((cur, s - cur))
    cur = max(cur, e)
print(f"{len(ev)} kernels, {len(marks)} markers; window {(t1 - t0) / 1e3:.1f} us, idle {sum(g for _, g in gaps) / 1e3:.1f} us "
      f"in {len(gaps)} gaps")
for g0, g in sorted(gaps, key=lambda x: -x[1])[:10]:
    before = [x for x in ev if x[1] <= g0][-1]
    after = [x for x in ev if x[0] >= g0 + g][0]
    print(f"  {g / 1e3:7.1f} us after {before[2]} (q{before[3]}) -> {after[2]} (q{after[3]})")
