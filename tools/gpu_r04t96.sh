# 96-wide 7-tap tiles (where the double-buffered chunk fits: dilation 1 / 3) after the staging
# work: vocoder alone and the bench, alternating with the 64-wide default.
set -o pipefail
O=gpurun_out/r04t96
mkdir -p $O
bash tools/codec_ab.sh X=1 RWKVTTS_CONV7_TN=96 X=1 RWKVTTS_CONV7_TN=96 > $O/codec_ab.txt 2>&1 || exit 1
grep -E "==|ms/batch|conv7|total" $O/codec_ab.txt
bash tools/bench_args_ab.sh "" "RWKVTTS_CONV7_TN=96" "" "RWKVTTS_CONV7_TN=96" "" "RWKVTTS_CONV7_TN=96" > $O/bench_ab.txt 2>&1; rc=$?
cat $O/bench_ab.txt; exit $rc
