set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
for a in "f16 mid" "bf16 mid" "f16 04b"; do echo "== $a"; timeout -k 10 200 python -u tools/persist_state_check.py $a || exit 1; done > $O/state_check.txt 2>&1; rc=$?; cat $O/state_check.txt; exit $rc
