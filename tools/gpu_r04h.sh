# Dispatch-time prefetches held back by a fixed time (RWKVTTS_PF_HOLD="w,late,s" in 10-ns ticks):
# decode A/B at B = 32 (tokens must not change).
set -o pipefail
O=gpurun_out/r04h3
mkdir -p $O
bash tools/db_env_ab.sh 2 "RWKVTTS_PF_HOLD=0,0,0" "RWKVTTS_PF_HOLD=100,0,0" "RWKVTTS_PF_HOLD=150,0,0" "RWKVTTS_PF_HOLD=200,0,0" "RWKVTTS_PF_HOLD=300,0,0" "RWKVTTS_PF_HOLD=150,150,0" "RWKVTTS_PF_HOLD=150,400,0" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
