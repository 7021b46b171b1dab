# Default 1-µs hold of the rkv / key weight streams: decode A/B against no hold and 0.8 / 1.2 µs,
# the bench against no hold, then the persistence / batching / full-length GPU tests.
set -o pipefail
O=gpurun_out/r04h4
mkdir -p $O
bash tools/db_env_ab.sh 2 "X=1" "RWKVTTS_PF_HOLD=0,0,0" "RWKVTTS_PF_HOLD=80,0,0" "RWKVTTS_PF_HOLD=120,0,0" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; [ $rc -eq 0 ] || exit $rc
bash tools/bench_args_ab.sh "" "RWKVTTS_PF_HOLD=0,0,0" "" "RWKVTTS_PF_HOLD=0,0,0" > $O/bench_ab.txt 2>&1; rc=$?
cat $O/bench_ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_ffn_persist.py tests/test_gpu_batching.py tests/test_gpu_emb_fusion.py tests/test_gpu_fulllength.py tests/test_gpu_manager.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; exit $rc
