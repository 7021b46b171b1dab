"""Decode-launch statistics of the B=32 decode-step kernels from a rocprofv3 --kernel-trace CSV of
a bench run: per kernel, the launches at the decode grid (prefill launches have
other grids or, for WKV, their own k_wkv6<..., true> symbol) with mean / median duration, and the
roofline fraction of the dominant kernel recomputed from them with the bench's algorithmic bytes.
Usage: decode_kernel_summary.py kernel_trace.csv out.json"""
import csv
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "rwkv-tts-rs_amd"))
from decode_kernels import DECODE  # noqa: E402
from bench import algorithmic_bytes, HBM_PEAK_GBS  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

rows = list(csv.DictReader(open(sys.argv[1])))
dur = {n: [] for n in DECODE}
syms = {n: set() for n in DECODE}
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rwkvtts::", "")
    g = int(r.get("Grid_Size", 0) or 0) or (int(r.get("Grid_Size_X", 1) or 1) * int(r.get("Grid_Size_Y", 1) or 1) *
                                            int(r.get("Grid_Size_Z", 1) or 1))
    for n, (prefixes, grid) in DECODE.items():
        if g == grid and any(name.startswith(p) for p in prefixes):
            dur[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            syms[n].add(name)
per, _ = algorithmic_bytes(W.DIMS_04B, 32, 8193)
out = {"source": os.path.basename(sys.argv[1]), "kernels": {}}
for n, d in dur.items():
    if not d:
        continue
    e = {"symbols": sorted(syms[n]), "launches": len(d), "mean_us": round(statistics.fmean(d), 3),
         "median_us": round(statistics.median(d), 3)}
    if n in per:
        e["algorithmic_bytes"] = per[n]
        e["frac_at_median"] = round(per[n] / (e["median_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
        e["frac_at_mean"] = round(per[n] / (e["mean_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    out["kernels"][n] = e
tot = {n: e["mean_us"] * e["launches"] for n, e in out["kernels"].items()}
if tot:
    out["dominant"] = max(tot, key=tot.get)
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out, indent=1))
