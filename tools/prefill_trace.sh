set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pf; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in ${PF_CHUNKS:-512 2048}; do
PF_CHUNK=$c timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t$c -o run -- python3 $R/tools/prefill_trace.py > $O/log$c.txt 2>&1 || exit 1
cat $O/log$c.txt | grep prefill
done
