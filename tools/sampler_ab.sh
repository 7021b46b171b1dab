# k_advance durations (rocprofv3 kernel trace of decode_bench, graph replay) with the certified
# sampler path and with the exact walk forced. Usage (GPU box): bash tools/sampler_ab.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/sab_${1:-cur}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/cert -o run -- python3 $R/tools/decode_bench.py 64 1 > $O/cert.log 2>&1 || { tail -5 $O/cert.log; exit 1; }
RWKVTTS_SAMPLER_EXACT=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/exact -o run -- python3 $R/tools/decode_bench.py 64 1 > $O/exact.log 2>&1 || { tail -5 $O/exact.log; exit 1; }
for m in cert exact; do
  f=$(find $O/$m -name "*kernel_trace.csv" | head -1)
  echo "== $m"; grep "rep " $O/$m.log
  python3 $R/tools/trace_summary.py $f advance
  python3 $R/tools/trace_summary.py $f wkv
done
