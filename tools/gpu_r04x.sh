# One-plane X staging in the persistent GEMM roles (LDS 36.6 -> 19.7 KB per workgroup: room beside
# a vocoder conv workgroup): decode alone and the bench (decode beside the vocoder), against the
# previous library (build/rev/base), with the 64- and 48-wide vocoder 7-tap tiles.
set -o pipefail
O=gpurun_out/r04x
mkdir -p $O
B=RWKVTTS_LIB=$PWD/build/abase/librwkvtts.so
bash tools/db_env_ab.sh 2 "X=1" "$B" > $O/decode_ab.txt 2>&1; rc=$?
cat $O/decode_ab.txt; [ $rc -eq 0 ] || exit $rc
bash tools/bench_args_ab.sh "" "$B" "RWKVTTS_CONV7_TN=48" "" "$B" "RWKVTTS_CONV7_TN=48" > $O/bench_ab.txt 2>&1; rc=$?
cat $O/bench_ab.txt; exit $rc
