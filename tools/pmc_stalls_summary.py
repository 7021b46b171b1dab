"""Per kernel class (name, grid) averages of the counters of tools/pmc_codec_stalls.sh's two
passes, with the derived ratios: wait / wave cycles, LDS-wait share, bank conflicts per LDS
instruction, MFMA and LDS instructions per wave. Usage: pass_a_dir pass_b_dir."""
import csv
import glob
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rwkvtts::", "")[:40], r.get("Grid_Size", ""))
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


a, b = load(sys.argv[1]), load(sys.argv[2])
print(f"{'kernel':40s} {'grid':>9s} {'wait/wv':>7s} {'ldsW/wv':>7s} {'lds/wv':>7s} {'valu/wv':>7s} {'bnkc/lds':>8s} "
      f"{'mfma/lds':>8s} {'fifo':>6s}")
for key in sorted(a, key=lambda k: -sum(a[k].get("SQ_WAVE_CYCLES", [0]))):
    c = {k: sum(v) / len(v) for k, v in a[key].items()}
    c.update({k: sum(v) / len(v) for k, v in b.get(key, {}).items()})
    wv = c.get("SQ_WAVE_CYCLES", 0) or 1
    lds = c.get("SQ_INSTS_LDS", 0) or 1
    print(f"{key[0]:40s} {key[1]:>9s} {c.get('SQ_WAIT_ANY', 0) / wv:7.3f} {c.get('SQ_WAIT_INST_LDS', 0) / wv:7.3f} "
          f"{c.get('SQ_ACTIVE_INST_LDS', 0) / wv:7.3f} {c.get('SQ_ACTIVE_INST_VALU', 0) / wv:7.3f} "
          f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / lds:8.3f} {c.get('SQ_INSTS_MFMA', 0) / lds:8.3f} "
          f"{c.get('SQ_LDS_DATA_FIFO_FULL', 0) / wv:6.3f}")
