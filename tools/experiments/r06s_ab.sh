# Round-6 A/B: the WKV -> Wo hand-off as row-indexed granules at multi-row decode steps vs the final
# library (ab_libs/fin): persistent-form / recovery / token GPU tests, decode_bench B = 8 / 32, bench x2.
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_ffn_persist.py tests/test_gpu_persist_recovery.py tests/test_gpu_generate.py tests/test_gpu_batching.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06s_tests.txt 2>&1 || { tail -30 gpurun_out/r06s_tests.txt; exit 1; }
tail -2 gpurun_out/r06s_tests.txt
LIBS="ab_libs/fin/librwkvtts.so rwkv-tts-rs_amd/rwkvtts/librwkvtts.so" BS="32 8" N=2 bash tools/db_multi_ab.sh 2>&1 | tee gpurun_out/r06s_db.txt || exit 1
for r in 1 2; do
bash tools/bench_ab.sh RWKVTTS_LIB=$R/ab_libs/fin/librwkvtts.so RWKVTTS_X=1 2>&1 | tee -a gpurun_out/r06s_bab.txt || exit 1
done
