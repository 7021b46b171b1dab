"""Summarise a RWKVTTS_DEBUG_STAMPS timeline= dump: per launch class, mean duration and the mean idle gap
before it (its start minus the previous launch's end), and the per-step totals."""
import sys
from collections import defaultdict

rows = [l.split() for l in open(sys.argv[1]) if not l.startswith("#")]
rows = [(int(a), b, float(c), float(d)) for a, b, c, d in rows]
dur, gap = defaultdict(list), defaultdict(list)
prev_end = None
for i, name, st, du in rows:
    dur[name].append(du)
    if prev_end is not None:
        gap[name].append(st - prev_end)
    prev_end = st + du
span = rows[-1][2] + rows[-1][3]
print(f"step span {span:.1f} us over {len(rows)} launches; sum of durations {sum(r[3] for r in rows):.1f} us")
for k in dur:
    g = gap.get(k, [0.0])
    print(f"{k:12s} n={len(dur[k]):3d} dur={sum(dur[k])/len(dur[k]):7.2f} gap_before={sum(g)/len(g):6.2f}  total={sum(dur[k])+sum(g):8.1f}")
