set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 300 bash -c 'for b in 1 8; do for e in "RWKVTTS_FFN_PERSIST=0 RWKVTTS_ATT_PERSIST=0" "RWKVTTS_FFN_PERSIST=5 RWKVTTS_ATT_PERSIST=5"; do echo -n "B=$b $e: "; env DB_B=$b $e timeout -k 10 120 python -u tools/decode_bench.py 128 1 | grep -oE "decode [0-9.]+ us/step" || exit 1; done; done' > $O/ab_small.txt 2>&1; rc=$?; cat $O/ab_small.txt; [ $rc -eq 0 ] || exit $rc
bash tools/timeline.sh RWKVTTS_FFN_PERSIST=5 > $O/timeline.txt 2>&1; rc=$?; cat $O/timeline.txt; [ $rc -eq 0 ] || exit $rc
TAG=r04h/t TEST_TIMEOUT=1500 bash tools/gpu_tests_then_bench.sh
