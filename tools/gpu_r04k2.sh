# Kernel-argument placement (HIP_FORCE_DEV_KERNARG) decode A/B, then attention-half stamps under
# the prefetch-order options.
set -o pipefail
O=gpurun_out/r04k2
mkdir -p $O
bash tools/db_env_ab.sh 2 "HIP_FORCE_DEV_KERNARG=0" "HIP_FORCE_DEV_KERNARG=1" "X=1" > $O/kernarg_ab.txt 2>&1; rc=$?
cat $O/kernarg_ab.txt; [ $rc -eq 0 ] || exit $rc
for v in 5 53; do echo "== ATT_PERSIST=$v"; RWKVTTS_ATT_PERSIST=$v timeout -k 10 120 python3 tools/ffn_stamps.py 32 att 32 2>&1 || exit 1; done > $O/att_opts.txt
cat $O/att_opts.txt
