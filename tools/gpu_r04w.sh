# Vocoder 7-tap tiles 48 wide (LDS room for a persistent decode workgroup beside them) vs 64: bench
# A/B (decode step beside the vocoder) and the vocoder alone.
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
bash tools/bench_args_ab.sh "" "RWKVTTS_CONV7_TN=48" "" "RWKVTTS_CONV7_TN=48" > $O/bench_ab.txt 2>&1; rc=$?
cat $O/bench_ab.txt; [ $rc -eq 0 ] || exit $rc
bash tools/codec_ab.sh RWKVTTS_CONV7_TN=64 RWKVTTS_CONV7_TN=48 > $O/codec_ab.txt 2>&1 || exit 1
grep -E "==|ms/batch|conv7" $O/codec_ab.txt
