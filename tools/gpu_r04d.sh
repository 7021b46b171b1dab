set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
for v in 11 13; do RWKVTTS_FFN_PERSIST=$v timeout -k 10 120 python -u tools/ffn_stamps.py 32 > $O/ffn_stamps$v.txt 2>&1; rc=$?; echo "== $v"; cat $O/ffn_stamps$v.txt; [ $rc -eq 0 ] || exit $rc; done
timeout -k 10 500 bash tools/db_env_ab.sh 2 RWKVTTS_FFN_PERSIST=0 RWKVTTS_FFN_PERSIST=5 RWKVTTS_FFN_PERSIST=9 RWKVTTS_FFN_PERSIST=11 RWKVTTS_FFN_PERSIST=13 RWKVTTS_FFN_PERSIST=15 > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc
