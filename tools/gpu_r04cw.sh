# k_conv staging by buffer loads into LDS (scalar offsets per chunk, out-of-range rows zeroed by
# the buffer range): the codec tests, then the vocoder alone and the bench against the previous
# library (build/abase), alternating.
set -o pipefail
O=gpurun_out/r04cw
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/codec_tests.log 2>&1
rc=$?; echo "CODEC TESTS EXIT $rc"; tail -3 $O/codec_tests.log; [ $rc -eq 0 ] || exit $rc
B=RWKVTTS_LIB=$PWD/build/abase/librwkvtts.so
bash tools/codec_ab.sh X=1 "$B" X=1 "$B" > $O/codec_ab.txt 2>&1 || exit 1
grep -E "==|ms/batch|total" $O/codec_ab.txt
bash tools/bench_args_ab.sh "" "$B" "" "$B" > $O/bench_ab.txt 2>&1; rc=$?
cat $O/bench_ab.txt; exit $rc
