set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
timeout -k 5 30 ./build/micro/bigarg || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_ffn_persist.py tests/test_gpu_emb_fusion.py -m gpu -x -v --timeout 150 --timeout-method thread > $O/persist_tests.log 2>&1; rc=$?; tail -12 $O/persist_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/db_env_ab.sh 2 "RWKVTTS_FFN_PERSIST=0 RWKVTTS_ATT_PERSIST=0" "RWKVTTS_LAYER_PERSIST=0" "RWKVTTS_LAYER_PERSIST=1 RWKVTTS_STEP_PERSIST=0" "RWKVTTS_STEP_PERSIST=1" > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/ffn_stamps.py 32 layer > $O/layer_stamps.txt 2>&1; cat $O/layer_stamps.txt
bash tools/gpu_r04n.sh
