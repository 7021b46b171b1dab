# Timing experiment: the LayerNorm rows without their shift-state load (results wrong; decode only).
set -o pipefail
O=gpurun_out/r04t
mkdir -p $O
bash tools/db_env_ab.sh 3 "RWKVTTS_DEBUG_LN=0" "RWKVTTS_DEBUG_LN=1" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
