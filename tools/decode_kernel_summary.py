"""Decode-launch statistics of the decode-step kernels from a rocprofv3 --kernel-trace CSV of a
bench run: per kernel, EVERY launch of its symbols (any row count: the
B=32 timed loop, the B=1 leg, prefill excluded by symbol / grid) and the subset that belongs to
the B=32 decode steps, with mean / median duration and the roofline fraction recomputed from the
B=32 subset with the bench's algorithmic bytes. The dominant kernel is picked as bench.py picks it:
the largest total time among the B=32 decode kernels with a byte model.

Row classes: the persistent attention launch's grid depends on the row count, the FFN launch's
does not (its LayerNorm blocks are padded to 32), so an FFN launch takes the class of the
attention launch before it in the trace (launches of one stream are ordered).
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
from decode_kernels import DECODE, ATT_GRIDS  # noqa: E402
from bench import algorithmic_bytes, HBM_PEAK_GBS  # noqa: E402
from rwkvtts import weights as W  # noqa: E402


def grid_of(r):
    g = int(r.get("Grid_Size", 0) or 0)
    return g or (int(r.get("Grid_Size_X", 1) or 1) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1))


def main(src, dst):
    rows = sorted(csv.DictReader(open(src)), key=lambda r: int(r["Start_Timestamp"]))
    allv = {n: [] for n in DECODE}
    b32 = {n: [] for n in DECODE}
    syms = {n: set() for n in DECODE}
    grids = {n: {} for n in DECODE}
    cls = None  # row class of the current decode step (from the last attention launch)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rwkvtts::", "")
        g = grid_of(r)
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for n, (prefixes, grid) in DECODE.items():
            if not any(name.startswith(p) for p in prefixes):
                continue
            if n == "att_persist":
                cls = ATT_GRIDS.get(g)  # rows of this step (None: not a known decode grid)
                row32 = g == grid
            elif n == "ffn_persist":
                row32 = g == grid and cls == 32
            else:
                row32 = g == grid
            if n == "ffn_persist" and cls is None:  # (no decode step seen yet)
                continue
            allv[n].append(us)
            grids[n][g] = grids[n].get(g, 0) + 1
            syms[n].add(name)
            if row32:
                b32[n].append(us)
            break
    per, _ = algorithmic_bytes(W.DIMS_04B, 32, 8193)
    out = {"source": os.path.basename(src), "kernels": {}}
    for n in DECODE:
        if not allv[n]:
            continue
        e = {"symbols": sorted(syms[n]), "launches_all_rows": len(allv[n]), "grids": grids[n],
             "mean_us_all_rows": round(statistics.fmean(allv[n]), 3)}
        d = b32[n]
        if d:
            e.update({"launches": len(d), "mean_us": round(statistics.fmean(d), 3),
                      "median_us": round(statistics.median(d), 3)})
            if n in per:
                e["algorithmic_bytes"] = per[n]
                e["frac_at_median"] = round(per[n] / (e["median_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
                e["frac_at_mean"] = round(per[n] / (e["mean_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
        out["kernels"][n] = e
    tot = {n: e["mean_us"] * e["launches"] for n, e in out["kernels"].items() if "launches" in e and n in per}
    if tot:
        out["dominant"] = max(tot, key=tot.get)
        out["dominant_rule"] = "largest B=32 total time among the decode kernels with a byte model (as bench.py)"
    from rwkvtts import _ffi
    out["build"] = _ffi.build_id()  # the library this trace was measured on (bench.py matches it)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
