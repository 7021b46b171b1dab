# Selected -m gpu tests (PYTEST_ARGS, default: the whole suite), then a short bench.
# Usage (from the repo root, via gpurun): TAG=r04a PYTEST_ARGS="tests/test_x.py" bash tools/gpu_tests_then_bench.sh
set -o pipefail
O=gpurun_out/${TAG:-tb}
mkdir -p $O
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -8 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python -u bench.py --steps ${STEPS:-5} --warmup 1 ${BENCH_ARGS:---no-cpu-baseline} > $O/bench.json 2> $O/bench.err
rc=$?; echo "BENCH EXIT $rc"
[ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms_per_step", d["ms_per_step"], "decode_step", d["decode_step_roofline"])
print("roofline", d["roofline"])
print("batch1", d.get("batch1"))
print("codec ms", d["codec_roofline"]["ms_per_batch"], "breakdown", d["breakdown_ms_per_batch"])
for k, v in d["kernels"].items(): print(" ", k, round(v["avg_us"], 2), v["launches"])
PY
