"""Per-launch HBM traffic of the B=32 decode-step kernels from the two rocprofv3 PMC passes
(FETCH_SIZE doubled for gfx950 wide streaming reads, WRITE_SIZE as is; MI355X_MICROARCH.md
HBM section), keyed by the bench's profile names. Usage: make_pmc_json.py fetch.csv write.csv out.json"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from decode_kernels import DECODE, match  # noqa: E402


def load(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rwkvtts::", "")
        acc[(name, int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return acc


f = load(sys.argv[1], "FETCH_SIZE")
w = load(sys.argv[2], "WRITE_SIZE")
out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, tools/lm_short.py (eager)",
       "correction": "FETCH_SIZE x2 (gfx950 reports half of 16-B/lane streaming reads); values in bytes per launch",
       "kernels": {}}
for name, (prefixes, grid) in DECODE.items():
    fv, syms = match(f, prefixes, grid)
    wv, _ = match(w, prefixes, grid)
    if not fv:
        print(f"WARNING: no FETCH_SIZE launches for {name} ({prefixes}, grid {grid})", file=sys.stderr)
        continue
    fb = 2 * 1024 * sum(fv) / len(fv)
    wb = 1024 * sum(wv) / max(len(wv), 1)
    out["kernels"][name] = {"symbols": syms, "grid": grid, "launches": len(fv),
                            "fetch_bytes": round(fb), "write_bytes": round(wb), "traffic_bytes": round(fb + wb)}
missing = [n for n in DECODE if n not in out["kernels"]]
if missing:
    print("WARNING: kernels missing from the PMC summary:", missing, file=sys.stderr)
# ratio to the bench's algorithmic bytes (SURVEY §8d model)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rwkv-tts-rs_amd"))
from bench import algorithmic_bytes  # noqa: E402
from rwkvtts import weights as W  # noqa: E402
per, _ = algorithmic_bytes(W.DIMS_04B, 32, 8193)
for name, e in out["kernels"].items():
    if name in per:
        e["algorithmic_bytes"] = per[name]
        e["traffic_over_algorithmic"] = round(e["traffic_bytes"] / per[name], 3)
from rwkvtts import _ffi  # noqa: E402
out["build"] = _ffi.build_id()  # the library these counters were measured on (bench.py matches it)
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out["kernels"], indent=1))
