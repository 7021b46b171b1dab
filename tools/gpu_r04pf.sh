# Vocoder L2 prefetch two chunks ahead (library build/pf): the codec tests on it, then the vocoder
# alone with the prefetch on / off and the in-tree library, alternating.
set -o pipefail
O=gpurun_out/r04pf
mkdir -p $O
L=$PWD/build/pf/librwkvtts.so
RWKVTTS_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/codec_tests.log 2>&1
rc=$?; echo "CODEC TESTS EXIT $rc"; tail -3 $O/codec_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/codec_ab.sh "RWKVTTS_LIB=$L" "RWKVTTS_LIB=$L RWKVTTS_CODEC_PF=0" "X=1" "RWKVTTS_LIB=$L" "RWKVTTS_LIB=$L RWKVTTS_CODEC_PF=0" > $O/codec_ab.txt 2>&1 || exit 1
grep -E "==|ms/batch|conv7|conv1|convT|total" $O/codec_ab.txt
