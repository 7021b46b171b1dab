"""MFMA utilisation per kernel from a rocprofv3 counter pass (SQ_VALU_MFMA_BUSY_CYCLES,
GRBM_GUI_ACTIVE) and a kernel-trace pass of the same command.
SQ_VALU_MFMA_BUSY_CYCLES adds 32 cycles per 32x32x16 (16 per 16x16x32) bf16 MFMA
(MI355X_MICROARCH.md), i.e. 1024 flops per busy cycle; the dense bf16 peak is 1024 SIMDs x 1024
flops per cycle. util = busy / (1024 SIMDs x kernel cycles); kernel cycles = duration x clock,
the clock taken from GRBM_GUI_ACTIVE (summed over the 8 XCDs) / duration of the same kernel class. Usage: pmc_dir kt_dir."""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rwkv-tts-rs_amd"))
from rwkvtts import _ffi  # noqa: E402

print(f"# build {_ffi.build_id()}")  # the library these counters were measured on (bench.py matches it)


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("rwkvtts::", "")
    return n[:48]


def find(d, pat):
    f = glob.glob(f"{d}/**/{pat}", recursive=True)
    return f[0] if f else None


pmc = find(sys.argv[1], "*counter_collection.csv")
kt = find(sys.argv[2], "*kernel_trace.csv")
cnt = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(pmc)):
    key = (short(r["Kernel_Name"]), r.get("Grid_Size", ""))
    cnt[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = defaultdict(list)
for r in csv.DictReader(open(kt)):
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])  # work-items
    key = (short(r["Kernel_Name"]), str(g))
    dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
print(f"{'kernel':48s} {'grid':>9s} {'n':>5s} {'avg_us':>8s} {'mfma_busy':>12s} {'clk_GHz':>7s} {'util':>6s} {'TFLOP/s':>8s}")
rows = []
for key, c in cnt.items():
    busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", [0])
    gui = c.get("GRBM_GUI_ACTIVE", [0])
    b = sum(busy) / len(busy)
    g = sum(gui) / len(gui)
    d = dur.get(key)
    if not d or b <= 0:
        continue
    t = sum(d) / len(d)
    clk = g / t / 1e9 if t > 0 else 0.0
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs (8 x the per-XCD cycle count)
    clk /= 8
    util = b / (1024 * g / 8) if g > 0 else 0.0
    rows.append((t * len(d), key, len(d), t, b, clk, util, b * 1024 / t / 1e12, g / 8))
for tot, key, n, t, b, clk, util, tf, _ in sorted(rows, reverse=True):
    print(f"{key[0]:48s} {key[1]:>9s} {n:5d} {t*1e6:8.1f} {b:12.4g} {clk:7.2f} {util:6.3f} {tf:8.1f}")
# time-weighted aggregate over the listed (MFMA-using) kernels
busy = sum(r[4] * r[2] for r in rows)
cyc = sum(1024 * r[8] * r[2] for r in rows)
secs = sum(r[0] for r in rows)
if cyc > 0:
    print(f"TOTAL mfma_util {busy / cyc:.4f} over {secs * 1e3:.2f} ms of MFMA kernels, "
          f"{busy * 1024 / secs / 1e12:.1f} TFLOP/s executed")
