"""Summarise a rocprofv3 --kernel-trace --stats directory: the kernels by total time,
and the copy / gather kernels (ATen index_select / gather, HIP blit copyBuffer) that the
serving launch path must not run.  python tools/kernel_census.py <rocprof out dir>"""
import csv
import glob
import os
import sys


def main(d: str) -> int:
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not stats:
        print("no kernel_stats.csv under", d)
        return 1
    rows = list(csv.DictReader(open(stats[0])))
    rows.sort(key=lambda r: -float(r.get("TotalDurationNs", 0)))
    tot = sum(float(r.get("TotalDurationNs", 0)) for r in rows)
    print(f"{'kernel':70s} {'calls':>7s} {'total ms':>10s} {'%':>6s}")
    for r in rows[:25]:
        t = float(r["TotalDurationNs"])
        print(f"{r['Name'][:70]:70s} {int(r['Calls']):7d} {t / 1e6:10.2f} {100 * t / tot:6.2f}")
    bad = [r for r in rows if any(k in r["Name"] for k in ("index_select", "indexSelect", "gather", "copyBuffer",
                                                             "index_fill", "CatArray", "elementwise_kernel"))]
    print("\ncopy / gather / elementwise kernels:")
    for r in bad:
        print(f"  {r['Name'][:110]:110s} calls {r['Calls']} total {float(r['TotalDurationNs']) / 1e6:.3f} ms")
    if not bad:
        print("  none")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
