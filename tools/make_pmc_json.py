"""Per-launch HBM traffic of the B=32 decode-step kernels from the two rocprofv3 PMC passes
(FETCH_SIZE doubled for gfx950 wide streaming reads, WRITE_SIZE as is; MI355X_MICROARCH.md
HBM section), keyed by the bench's profile names. Usage: make_pmc_json.py fetch.csv write.csv out.json"""
import csv
import json
import os
import sys
from collections import defaultdict

# (kernel symbol prefix, grid size) of each decode-step launch at 32 rows (0.4B dims)
DECODE = {
    "gemm_rkv_lora": ("k_gemm2<2, 8, 0, false, 1, 2, false>", 54272),
    "gemm_ffn_key": ("k_gemm2<2, 8, 0, false, 1, 0, false>", 65536),
    "gemm_wo": ("k_gemm2<2, 4, 0, false, 1, 0, false>", 32768),
    "gemm_ffn_value": ("k_gemm2<2, 8, 1, false, 4, 0, false>", 65536),
    "wkv": ("k_wkv6<false>", 131072),
    "ln_mix_att": ("k_ln1024<false, 1, 6, 16>", 8192),
    "ln_mix_ffn": ("k_ln1024<false, 1, 1, 8>", 8192),
}


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
for name, key in DECODE.items():
    if key in f:
        fb = 2 * 1024 * sum(f[key]) / len(f[key])
        wb = 1024 * sum(w.get(key, [0.0])) / max(len(w.get(key, [1])), 1)
        out["kernels"][name] = {"symbol": key[0], "grid": key[1], "launches": len(f[key]),
                                "fetch_bytes": round(fb), "write_bytes": round(wb), "traffic_bytes": round(fb + wb)}
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
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out["kernels"], indent=1))
