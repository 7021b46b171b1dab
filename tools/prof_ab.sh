# Kernel-trace A/B of the decode microbenchmark: per-kernel duration and preceding gap for each
# environment setting given (e.g. "X=1" "DB_FORMS=1"). Usage: bash tools/prof_ab.sh ENV...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for e in "$@"; do
  i=$((i+1)); O=$R/gpurun_out/profab_$i; mkdir -p $O
  echo "== $e"
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 $R/tools/decode_bench.py 48 1 > $O/log.txt 2>&1 || { tail -5 $O/log.txt; exit 1; }
  grep "rep 0" $O/log.txt
  f=$(find $O -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/gap_summary.py $f | tee $O/summary.txt
done
