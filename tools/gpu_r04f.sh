set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ffn_persist.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/persist_tests.log 2>&1; rc=$?; tail -8 $O/persist_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/ffn_stamps.py 32 att > $O/att_stamps.txt 2>&1; rc=$?; cat $O/att_stamps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/db_env_ab.sh 2 "RWKVTTS_FFN_PERSIST=0 RWKVTTS_ATT_PERSIST=0" "RWKVTTS_FFN_PERSIST=5 RWKVTTS_ATT_PERSIST=0" "RWKVTTS_FFN_PERSIST=0 RWKVTTS_ATT_PERSIST=5" "RWKVTTS_FFN_PERSIST=5 RWKVTTS_ATT_PERSIST=5" "RWKVTTS_FFN_PERSIST=5 RWKVTTS_ATT_PERSIST=1" > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc
