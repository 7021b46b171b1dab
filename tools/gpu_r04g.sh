set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ffn_persist.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/persist_tests.log 2>&1; rc=$?; tail -3 $O/persist_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 5 21; do RWKVTTS_ATT_PERSIST=$v timeout -k 10 120 python -u tools/ffn_stamps.py 32 att > $O/att_stamps$v.txt 2>&1; rc=$?; echo "== $v"; cat $O/att_stamps$v.txt; [ $rc -eq 0 ] || exit $rc; done
timeout -k 10 600 bash tools/db_env_ab.sh 2 "RWKVTTS_FFN_PERSIST=0 RWKVTTS_ATT_PERSIST=0" "RWKVTTS_FFN_PERSIST=5 RWKVTTS_ATT_PERSIST=5" "RWKVTTS_FFN_PERSIST=5 RWKVTTS_ATT_PERSIST=21" "RWKVTTS_FFN_PERSIST=5 RWKVTTS_ATT_PERSIST=37" "RWKVTTS_FFN_PERSIST=5 RWKVTTS_ATT_PERSIST=53" "RWKVTTS_FFN_PERSIST=7 RWKVTTS_ATT_PERSIST=21" > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc
