"""Per-kernel totals of a rocprofv3 --kernel-trace CSV, over the launches after the first
`skip` fraction (default: the second half, e.g. the second of two identical runs).
Usage: trace_kernels.py kernel_trace.csv [skip_fraction]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
rows = rows[int(len(rows) * skip):]
tot, cnt = defaultdict(float), defaultdict(int)
for r in rows:
    g = r.get("Grid_Size") or str(int(r.get("Grid_Size_X", 1) or 1) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1))
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rwkvtts::", "")[:60] + " g" + g
    tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[k] += 1
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"span {span:.1f} us, kernel time {sum(tot.values()):.1f} us over {len(rows)} launches")
for k in sorted(tot, key=lambda k: -tot[k])[:25]:
    print(f"{tot[k]:10.1f} us {cnt[k]:6d} x {tot[k] / cnt[k]:8.2f} us  {k}")
