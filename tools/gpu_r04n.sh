set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 5 --no-cpu-baseline --no-batch1 > $O/b_gt.json 2> $O/b_gt.err || { tail $O/b_gt.err; exit 1; }
timeout -k 10 600 python -u bench.py --steps 5 --no-cpu-baseline --no-batch1 --no-graph-timing > $O/b_eager.json 2> $O/b_eager.err || { tail $O/b_eager.err; exit 1; }
python3 - <<'PY'
import json
for f in ("b_gt", "b_eager"):
    d = json.loads(open(f"gpurun_out/r04n/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["decode_step_roofline"]["ms_per_decode_step"], d["roofline"]["kernel"], d["roofline"]["avg_us"], d["roofline"]["frac"])
    print("  ", {k: (v["launches"], round(v["avg_us"], 2)) for k, v in d["kernels"].items()})
PY
bash tools/gpu_profiles.sh r04b
