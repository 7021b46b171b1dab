# HBM traffic of the vocoder kernels (codec_bench.py 32 x 512): FETCH_SIZE and WRITE_SIZE passes
# (MI355X_MICROARCH.md: FETCH_SIZE x 2 on gfx950), per kernel class. Output under gpurun_out/ctraf/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ctraf
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 $R/tools/codec_bench.py 32 512 > $O/f.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 $R/tools/codec_bench.py 32 512 > $O/w.log 2>&1
rc=$?; echo "PMC EXIT $rc"
python3 - $O <<'PY'
import csv, glob, sys
from collections import defaultdict
O = sys.argv[1]
def load(d, name):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    acc = defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != name: continue
        k = (r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rwkvtts::", "")[:44], r.get("Grid_Size", ""))
        acc[k].append(float(r["Counter_Value"]))
    return acc
fe, wr = load(O + "/f", "FETCH_SIZE"), load(O + "/w", "WRITE_SIZE")
print(f"{'kernel':44s} {'grid':>10s} {'n':>4s} {'fetch GB/launch':>16s} {'write GB/launch':>16s}")
for k in sorted(fe, key=lambda k: -sum(fe[k])):
    n = len(fe[k]) // 4 or 1  # codec_bench runs 1 + 3 + 1 batches; per-launch mean
    f = 2 * sum(fe[k]) / len(fe[k]) * 1024 / 1e9   # KB -> GB, x2 gfx950 correction
    w = sum(wr.get(k, [0])) / max(len(wr.get(k, [1])), 1) * 1024 / 1e9
    print(f"{k[0]:44s} {k[1]:>10s} {len(fe[k]):4d} {f:16.3f} {w:16.3f}")
PY
