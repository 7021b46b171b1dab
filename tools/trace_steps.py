"""Per-step kernel time from a rocprofv3 kernel-trace CSV: steps are delimited by k_advance launches.
Prints, for the first N steps, the step's span and its kernels aggregated by name.
Usage: trace_steps.py kernel_trace.csv|dir [N]"""
import csv
import sys
from collections import defaultdict

import glob
import os
src = sys.argv[1]
if os.path.isdir(src):
    src = sorted(glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True))[0]
rows = sorted(csv.DictReader(open(src)), key=lambda r: int(r["Start_Timestamp"]))
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4
rows = [r for r in rows if "rwkvtts" in r["Kernel_Name"]]
step, cur = [], []
for r in rows:
    cur.append(r)
    if "k_advance" in r["Kernel_Name"]:
        step.append(cur)
        cur = []
for i, s in enumerate(step[:N]):
    t0, t1 = int(s[0]["Start_Timestamp"]), int(s[-1]["End_Timestamp"])
    agg = defaultdict(lambda: [0, 0.0])
    for r in s:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rwkvtts::", "")
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    busy = sum(v[1] for v in agg.values())
    print(f"step {i}: {len(s)} launches, span {(t1 - t0) / 1000:.1f} us, busy {busy:.1f} us")
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:8]:
        print(f"    {k[:60]:60s} n={n:4d} total={us:9.1f} us avg={us / n:8.2f}")
