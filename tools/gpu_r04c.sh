# persistent FFN: per-block stamps, TL timelines of both FFN forms, variant A/B
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 120 python -u tools/ffn_stamps.py 32 > $O/ffn_stamps.txt 2>&1; rc=$?; cat $O/ffn_stamps.txt; [ $rc -eq 0 ] || exit $rc
RWKVTTS_FFN_PERSIST=3 timeout -k 10 120 python -u tools/ffn_stamps.py 32 > $O/ffn_stamps3.txt 2>&1; rc=$?; cat $O/ffn_stamps3.txt; [ $rc -eq 0 ] || exit $rc
bash tools/timeline.sh RWKVTTS_FFN_PERSIST=0 RWKVTTS_FFN_PERSIST=1 > $O/timeline.txt 2>&1; rc=$?; cat $O/timeline.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash tools/db_env_ab.sh 2 RWKVTTS_FFN_PERSIST=0 RWKVTTS_FFN_PERSIST=1 RWKVTTS_FFN_PERSIST=3 RWKVTTS_FFN_PERSIST=5 RWKVTTS_FFN_PERSIST=7 > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc
