# Round-6 A/B: k_gemm_wide variants (LDS-only barriers; three workgroups per CU) vs the tree and
# the round-6 head library: prefill kernel traces.
set -o pipefail
for v in wbar wocc; do
  bash tools/prefill_lib_trace.sh r06o_$v ab_libs/head/librwkvtts.so ab_libs/$v/librwkvtts.so > /dev/null || exit 1
  grep -E "==|prefill_ms|gemm|wkv6" gpurun_out/pft_r06o_$v/summary.txt
done
bash tools/prefill_lib_trace.sh r06o_tree ab_libs/head/librwkvtts.so rwkv-tts-rs_amd/rwkvtts/librwkvtts.so > /dev/null || exit 1
grep -E "==|prefill_ms|gemm|wkv6" gpurun_out/pft_r06o_tree/summary.txt
