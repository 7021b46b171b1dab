# Round profiles: rocprofv3 kernel-trace --stats of a bench run (the bench's default command minus
# the CPU baseline) + separate PMC passes (FETCH_SIZE, WRITE_SIZE) on the short LM workload.
# Usage: gpu_profiles.sh TAG. Outputs under gpurun_out/prof_TAG/; then, on the CPU side:
#   python3 tools/decode_kernel_summary.py <trace>/..._kernel_trace.csv profiles/TAG_decode_kernels.json
#   python3 tools/make_pmc_json.py <fetch csv> <write csv> profiles/TAG_pmc_traffic.json
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_${1:-r04}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 $R/bench.py --no-cpu-baseline > $O/bench_trace.log 2>&1 || exit 1
export LM_GRAPHS=0
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/tools/lm_short.py > $O/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/tools/lm_short.py > $O/write.log 2>&1 || exit 1
echo PROFILES_OK; find $O -name "*.csv" | head -20
