"""Summarise a rocprofv3 kernel-trace CSV: per kernel name, dispatch durations (us)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
d = defaultdict(list)
for r in rows:
    d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for k, v in d.items():
    if pat in k:
        print(f"{k[:70]:70s} n={len(v):6d} avg={sum(v)/len(v):9.2f} min={min(v):8.2f}")
        if len(sys.argv) > 3:
            print("   ", " ".join(f"{x:.1f}" for x in v[: int(sys.argv[3])]))
