# Vocoder 7-tap tile rule (48 wide only where it frees room for a decode workgroup) vs 64 / 48
# everywhere: three alternating bench triples, then the vocoder alone.
set -o pipefail
O=gpurun_out/r04z
mkdir -p $O
bash tools/bench_args_ab.sh "" "RWKVTTS_CONV7_TN=64" "RWKVTTS_CONV7_TN=48" "" "RWKVTTS_CONV7_TN=64" "RWKVTTS_CONV7_TN=48" "" "RWKVTTS_CONV7_TN=64" "RWKVTTS_CONV7_TN=48" > $O/bench_ab.txt 2>&1; rc=$?
cat $O/bench_ab.txt; [ $rc -eq 0 ] || exit $rc
bash tools/codec_ab.sh X=1 RWKVTTS_CONV7_TN=64 > $O/codec_ab.txt 2>&1 || exit 1
grep -E "==|ms/batch|conv7|total" $O/codec_ab.txt
