# End-of-round check: smoke(), the whole -m gpu suite, the bench of record (10 steps, CPU
# baseline, B=1 leg), then the rocprof / PMC profiles of the bench command (tag r04d).
set -o pipefail
O=gpurun_out/r04fin3
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
TAG=r04fin3/t TEST_TIMEOUT=900 NO_BENCH=1 bash tools/gpu_tests_then_bench.sh || exit 1
timeout -k 10 600 python -u bench.py --steps 10 --warmup 1 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 1200 $O/bench.json
bash tools/gpu_profiles.sh r04f
