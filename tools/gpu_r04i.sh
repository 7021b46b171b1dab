set -o pipefail
O=gpurun_out/r04i
mkdir -p $O
TAG=r04i/t TEST_TIMEOUT=1500 bash tools/gpu_tests_then_bench.sh
