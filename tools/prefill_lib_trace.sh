# Prefill kernels of two library builds: rocprofv3 kernel trace of tools/prefill_trace.py (the bench's 32
# prompts, token_chunk_size 2048: one prefill step) per library, per-kernel totals of the second run
# (tools/trace_kernels.py). Usage: bash tools/prefill_lib_trace.sh TAG LIB_A LIB_B
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:?TAG}; O=$R/gpurun_out/pft_$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
n=0
for L in "$2" "$3"; do
  n=$((n + 1))
  RWKVTTS_LIB=$R/$L PF_CHUNK=2048 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t$n -o run -- python3 $R/tools/prefill_trace.py > $O/log$n.txt 2>&1 || exit 1
  KT=$(find $O/t$n -name "*kernel_trace.csv" | head -1)
  { echo "== $L"; grep prefill $O/log$n.txt; python3 $R/tools/trace_kernels.py $KT 0.5 | head -14; } >> $O/summary.txt
  rm -f $KT
done
cat $O/summary.txt
