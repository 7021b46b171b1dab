set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
for a in "f16 mid" "f16 04b"; do echo "== $a"; timeout -k 10 200 python -u tools/persist_state_check.py $a || exit 1; done > $O/state_check.txt 2>&1; rc=$?; cat $O/state_check.txt; [ $rc -eq 0 ] || exit $rc
TAG=r04k/t TEST_TIMEOUT=1500 bash tools/gpu_tests_then_bench.sh
