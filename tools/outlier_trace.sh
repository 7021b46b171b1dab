# Decode-launch outliers beside the vocoder: rocprofv3 --kernel-trace of a short pipelined bench
# (2 timed batches: the vocoder of each beside the next one's decode), then tools/outlier_attrib.py
# on the box; only the report is kept (the trace CSV is deleted). Usage: bash tools/outlier_trace.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-outl}
O=$R/gpurun_out/outl_$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-batch1 --no-graph-timing > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
KT=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/outlier_attrib.py $KT 4 25 > $O/${T}_outliers.txt || exit 1
rm -f $KT
head -60 $O/${T}_outliers.txt
