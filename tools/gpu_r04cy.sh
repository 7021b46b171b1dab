# k_conv_out window loads batched (8 pieces per thread in flight): the codec tests, then the vocoder
# alone against the previous library (build/abase2), alternating.
set -o pipefail
set -o pipefail
O=gpurun_out/r04cy
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/codec_tests.log 2>&1
rc=$?; echo "CODEC TESTS EXIT $rc"; tail -3 $O/codec_tests.log; [ $rc -eq 0 ] || exit $rc
B=RWKVTTS_LIB=$PWD/build/abase2/librwkvtts.so
bash tools/codec_ab.sh X=1 "$B" X=1 "$B" > $O/codec_ab.txt 2>&1 || exit 1
grep -E "==|ms/batch|total" $O/codec_ab.txt
exit 0
cat $O/bench_ab.txt; exit $rc
