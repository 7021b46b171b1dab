# One launch per layer with the FFN roles' weight streams held back (FFN_PERSIST opts: 4 = key
# weights after the LN wait, 1 = value weights after the LN rows) vs two launches per layer.
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
bash tools/db_env_ab.sh 2 "RWKVTTS_LAYER_PERSIST=0" "RWKVTTS_LAYER_PERSIST=1" "RWKVTTS_LAYER_PERSIST=1 RWKVTTS_FFN_PERSIST=13" "RWKVTTS_LAYER_PERSIST=1 RWKVTTS_FFN_PERSIST=15" "RWKVTTS_LAYER_PERSIST=1 RWKVTTS_FFN_PERSIST=7" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
