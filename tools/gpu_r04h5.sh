# FFN value weights held (4th field of RWKVTTS_PF_HOLD) on top of the default 1-us rkv / key hold.
set -o pipefail
O=gpurun_out/r04h6
mkdir -p $O
bash tools/db_env_ab.sh 2 "X=1" "RWKVTTS_PF_HOLD=100,0,0,0,0" "RWKVTTS_PF_HOLD=100,0,0,0,200" "RWKVTTS_PF_HOLD=150,0,0,0,100" "RWKVTTS_PF_HOLD=70,0,0,0,100" "RWKVTTS_PF_HOLD=150,0,0,0,150" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
