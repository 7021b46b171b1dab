# Round-6 A/B: k_gemm_wide with plain (not write-through) slab stores vs the tree: prefill traces.
set -o pipefail
for r in 1 2; do
bash tools/prefill_lib_trace.sh r06p_$r rwkv-tts-rs_amd/rwkvtts/librwkvtts.so ab_libs/wnowt/librwkvtts.so > /dev/null || exit 1
grep -E "==|prefill_ms|gemm|wkv6|ln1024" gpurun_out/pft_r06p_$r/summary.txt
done
