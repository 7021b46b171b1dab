# Round profiles: rocprofv3 kernel-trace --stats of a bench run (the bench's default command minus
# the CPU baseline) + separate PMC passes (FETCH_SIZE, WRITE_SIZE) on the short LM workload, then
# the summaries (decode-launch statistics, PMC traffic per decode kernel) made on the box; the
# large per-launch CSVs are deleted (gpurun copies back <= 64 MiB). Usage: gpu_profiles.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r04}
O=$R/gpurun_out/prof_$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 $R/bench.py --no-cpu-baseline > $O/bench_trace.log 2>&1 || { tail -20 $O/bench_trace.log; exit 1; }
tail -c 400 $O/bench_trace.log
export LM_GRAPHS=0
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/tools/lm_short.py > $O/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/tools/lm_short.py > $O/write.log 2>&1 || exit 1
cd $R
KT=$(find $O/trace -name "*kernel_trace.csv" | head -1)
KS=$(find $O/trace -name "*kernel_stats.csv" | head -1)
FC=$(find $O/fetch -name "*counter_collection.csv" | head -1)
WC=$(find $O/write -name "*counter_collection.csv" | head -1)
cp $KS $O/${T}_bench_kernel_stats.csv
python3 tools/decode_kernel_summary.py $KT $O/${T}_decode_kernels.json > /dev/null || exit 1
python3 tools/make_pmc_json.py $FC $WC $O/${T}_pmc_traffic.json > /dev/null || exit 1
python3 tools/trace_kernels.py $KT 0.5 > $O/${T}_trace_top.txt || exit 1
rm -f $KT $FC $WC
echo PROFILES_OK; ls -la $O
