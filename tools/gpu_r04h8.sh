# Poll sleep (persist option bit 1) with the weight-stream hold: decode A/B at B = 32.
set -o pipefail
O=gpurun_out/r04h9
mkdir -p $O
bash tools/db_env_ab.sh 4 "X=1" "RWKVTTS_ATT_PERSIST=1" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
