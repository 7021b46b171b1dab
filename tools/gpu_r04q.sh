# Channel-blocked vocoder planes: the codec tests and a vocoder A/B first, then the whole -m gpu suite.
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/codec_tests.log 2>&1
rc=$?; echo "CODEC TESTS EXIT $rc"; tail -5 $O/codec_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/codec_ab.sh RWKVTTS_CODEC_BLK=1 RWKVTTS_CODEC_BLK=0 RWKVTTS_CODEC_BLK=1 RWKVTTS_CODEC_BLK=0 > $O/codec_ab.txt 2>&1 || exit 1
grep -E "==|ms/batch" $O/codec_ab.txt
TAG=r04q/t TEST_TIMEOUT=900 NO_BENCH=1 bash tools/gpu_tests_then_bench.sh
