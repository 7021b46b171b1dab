# Round-6 A/B: wide prefill GEMMs (k_gemm_wide) vs the round-6 head library: bitwise GPU tests,
# prefill kernel trace, bench.py --steps 3 A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_batching.py tests/test_gpu_generate.py tests/test_gpu_f16_range.py tests/test_gpu_quant.py tests/test_gpu_emb_fusion.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06n_tests.txt 2>&1 || { tail -30 gpurun_out/r06n_tests.txt; exit 1; }
tail -2 gpurun_out/r06n_tests.txt
bash tools/prefill_lib_trace.sh r06n ab_libs/head/librwkvtts.so rwkv-tts-rs_amd/rwkvtts/librwkvtts.so > /dev/null || exit 1
grep -vE "^W2026|^\s*$" gpurun_out/pft_r06n/summary.txt
bash tools/bench_ab.sh RWKVTTS_LIB=$R/ab_libs/head/librwkvtts.so RWKVTTS_X=1 RWKVTTS_LIB=$R/ab_libs/head/librwkvtts.so RWKVTTS_X=1 2>&1 | tee gpurun_out/r06n_bab.txt
