"""Per-kernel-family summary of a rocprofv3 --pmc counter collection (tools/pmc_bench.sh):
dispatches, mean GRBM_GUI_ACTIVE cycles (rocprofv3 sums them over the 8 XCDs), MFMA utilisation =
SQ_VALU_MFMA_BUSY_CYCLES (MFMA cycles summed over all SIMDs) / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs),
wave cycles waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES), issuing (SQ_ACTIVE_INST_ANY / ...), LDS
bank-conflict cycles. (Kernels are serialised by the counter collection.)

python tools/pmc_summary.py gpurun_out/pmc_bench/p1/run_counter_collection.csv [--out f.csv]
"""
import argparse
import csv
import re
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("counters")
ap.add_argument("--out", default="")
ap.add_argument("--simds", type=int, default=1024)
ap.add_argument("--xcds", type=int, default=8)
a = ap.parse_args()
per = defaultdict(lambda: defaultdict(float))  # (dispatch id) -> counter -> value
name = {}
for r in csv.DictReader(open(a.counters)):
    d = r.get("Dispatch_Id") or r.get("Correlation_Id")
    per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    name[d] = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:80]
fam = defaultdict(lambda: defaultdict(float))
for d, cs in per.items():
    f = fam[name[d]]
    f["n"] += 1
    for k, v in cs.items():
        f[k] += v
rows = []
for k, f in fam.items():
    gui = f["GRBM_GUI_ACTIVE"] or 1.0
    wave = f["SQ_WAVE_CYCLES"] or 1.0
    rows.append({"kernel": k, "dispatches": int(f["n"]), "gui_cycles_mean": round(gui / f["n"]),
                 "mfma_util": round(f["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui / a.xcds * a.simds), 3),
                 "wait_any": round(f["SQ_WAIT_ANY"] / wave, 3), "issuing": round(f["SQ_ACTIVE_INST_ANY"] / wave, 3),
                 "wait_lds": round(f["SQ_WAIT_INST_LDS"] / wave, 3), "lds_conflict_cycles": int(f["SQ_LDS_BANK_CONFLICT"])})
rows.sort(key=lambda r: -r["gui_cycles_mean"] * r["dispatches"])
for r in rows[:30]:
    print(f"{r['kernel']:80s} {r['dispatches']:4d} {r['gui_cycles_mean']:9d} mfma {r['mfma_util']:.3f} "
          f"wait {r['wait_any']:.2f} issue {r['issuing']:.2f} lds {r['wait_lds']:.2f} conf {r['lds_conflict_cycles']}")
if a.out:
    with open(a.out, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
