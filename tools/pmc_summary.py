"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE counter CSVs per kernel (per-dispatch average,
FETCH_SIZE doubled per MI355X_MICROARCH.md: gfx950 reports half of wide streaming reads)."""
import csv
import sys
from collections import defaultdict


def load(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rwkvtts::", "")
        acc[(name, r.get("Grid_Size", ""))].append(float(r["Counter_Value"]))
    return acc


f = load(sys.argv[1], "FETCH_SIZE")
w = load(sys.argv[2], "WRITE_SIZE")
print(f"{'kernel':38s} {'grid':>9s} {'n':>6s} {'fetch KB x2':>12s} {'write KB':>10s}")
for key in sorted(f, key=lambda k: -sum(f[k]) / len(f[k]) * len(f[k])):
    n = len(f[key])
    fk = 2 * sum(f[key]) / n
    wk = sum(w.get(key, [0])) / max(len(w.get(key, [1])), 1)
    print(f"{key[0][:38]:38s} {key[1]:>9s} {n:6d} {fk:12.1f} {wk:10.1f}")
