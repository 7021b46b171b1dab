# Speculative shift-row loads in the LayerNorm rows: decode A/B (RWKVTTS_DEBUG_LN=2 turns them off;
# tokens must match), then the decode / batching / persistence GPU tests.
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
bash tools/db_env_ab.sh 3 "RWKVTTS_DEBUG_LN=0" "RWKVTTS_DEBUG_LN=2" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_ffn_persist.py tests/test_gpu_batching.py tests/test_gpu_emb_fusion.py tests/test_gpu_generate.py tests/test_gpu_forward.py tests/test_gpu_fulllength.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log; exit $rc
