set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
TAG=r04p/t TEST_TIMEOUT=1500 BENCH_ARGS=" " STEPS=10 bash tools/gpu_tests_then_bench.sh || exit 1
bash tools/gpu_profiles.sh r04c
