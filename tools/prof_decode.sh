# rocprofv3 kernel trace of the decode microbenchmark; per-kernel durations and gaps.
# Usage (GPU box): bash tools/prof_decode.sh TAG [S]
set -o pipefail
TAG=${1:-cur}; S=${2:-32}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 $R/tools/decode_bench.py $S 1 > $O/log.txt 2>&1 || { tail -5 $O/log.txt; exit 1; }
f=$(find $O -name "*kernel_trace.csv" | head -1)
python3 $R/tools/gap_summary.py $f | tee $O/summary.txt
