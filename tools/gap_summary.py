"""From a rocprofv3 kernel-trace CSV: per-kernel average duration and the average idle gap
that precedes each kernel (start - previous end on the same queue), restricted to the
steady-state decode window (dispatches between the first and last k_advance)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adv = [i for i, r in enumerate(rows) if "k_advance" in r["Kernel_Name"]]
lo, hi = adv[len(adv) // 4], adv[-2]
dur, gap = defaultdict(list), defaultdict(list)
for i in range(lo + 1, hi + 1):
    r, p = rows[i], rows[i - 1]
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rwkvtts::", "")[:34]
    gsz = r.get("Grid_Size") or r.get("Grid_Size_X") or ""
    k = f"{k} g{gsz}"
    dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    gap[k].append((int(r["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1000)
steps = sum(1 for i in range(lo + 1, hi + 1) if "k_advance" in rows[i]["Kernel_Name"])
tot_d = sum(sum(v) for v in dur.values()) / steps
tot_g = sum(sum(v) for v in gap.values()) / steps
span = (int(rows[hi]["End_Timestamp"]) - int(rows[lo]["End_Timestamp"])) / 1000 / steps
print(f"steps={steps} per-step: span={span:.1f}us kernels={tot_d:.1f}us gaps={tot_g:.1f}us")
for k in dur:
    n = len(dur[k]) / steps
    print(f"{k:44s} per-step n={n:5.1f} avg_dur={sum(dur[k])/len(dur[k]):7.2f} avg_gap={sum(gap[k])/len(gap[k]):6.2f}")
