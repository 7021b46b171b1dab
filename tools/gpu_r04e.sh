set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ffn_persist.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/persist_tests.log 2>&1; rc=$?; tail -3 $O/persist_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 11 15; do RWKVTTS_FFN_PERSIST=$v timeout -k 10 120 python -u tools/ffn_stamps.py 32 > $O/ffn_stamps$v.txt 2>&1; rc=$?; echo "== $v"; cat $O/ffn_stamps$v.txt; [ $rc -eq 0 ] || exit $rc; done
timeout -k 10 500 bash tools/db_env_ab.sh 2 RWKVTTS_FFN_PERSIST=0 RWKVTTS_FFN_PERSIST=1 RWKVTTS_FFN_PERSIST=5 RWKVTTS_FFN_PERSIST=11 RWKVTTS_FFN_PERSIST=15 > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc
