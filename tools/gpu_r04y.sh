# Vocoder 7-tap tiles 48 vs 64 wide beside the decode: four alternating bench pairs.
set -o pipefail
O=gpurun_out/r04y
mkdir -p $O
bash tools/bench_args_ab.sh "" "RWKVTTS_CONV7_TN=48" "" "RWKVTTS_CONV7_TN=48" "" "RWKVTTS_CONV7_TN=48" "" "RWKVTTS_CONV7_TN=48" > $O/bench_ab.txt 2>&1; rc=$?
cat $O/bench_ab.txt; exit $rc
