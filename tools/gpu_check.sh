# GPU check: full -m gpu suite, then a short bench (no CPU baseline). Each step time-limited.
# Extra pytest arguments (e.g. --deselect ...) come from $PYTEST_EXTRA.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $PYTEST_EXTRA > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?; echo "BENCH EXIT $rc"
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_quick.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms_per_step", d["ms_per_step"], "decode_step", d["decode_step_roofline"])
print("codec ms", d["codec_roofline"]["ms_per_batch"])
for k, v in d["kernels"].items(): print(" ", k, round(v["avg_us"], 2), v["launches"])
PY
exit $rc
