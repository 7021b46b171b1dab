# Copy one gpu_round.sh session's summaries into profiles/ (tracked): TAG_bench.json, TAG_gpu_suite.txt,
# TAG_smoke.txt, TAG_fulllength_report.json, TAG_bench_kernel_stats.csv, TAG_decode_kernels.json,
# TAG_pmc_traffic.json, TAG_trace_top.txt, TAG_mfma_codec.txt, TAG_mfma_lm.txt (whichever exist).
# Usage: bash tools/keep_profiles.sh TAG
T=${1:?usage: keep_profiles.sh TAG}
G=gpurun_out
cp_if() { [ -f "$1" ] && cp "$1" "profiles/$2" && echo "profiles/$2"; }
cp_if $G/$T/bench.json ${T}_bench.json
cp_if $G/$T/gpu_suite.txt ${T}_gpu_suite.txt
cp_if $G/$T/smoke.txt ${T}_smoke.txt
cp_if $G/$T/fulllength_report.json ${T}_fulllength_report.json
for f in bench_kernel_stats.csv decode_kernels.json pmc_traffic.json trace_top.txt; do cp_if $G/prof_$T/${T}_$f ${T}_$f; done
cp_if $G/mfma_$T/codec_summary.txt ${T}_mfma_codec.txt
cp_if $G/mfma_$T/lm_summary.txt ${T}_mfma_lm.txt
true
