set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
for e in "RWKVTTS_ATT_PERSIST=5 RWKVTTS_FFN_PERSIST=0" "RWKVTTS_ATT_PERSIST=0 RWKVTTS_FFN_PERSIST=5"; do
echo "== $e"
env $e timeout -k 10 400 python -u -m pytest tests/test_gpu_manager.py -m gpu -x -q -k config4 --timeout 300 --timeout-method thread -s > $O/m.log 2>&1; rc=$?; grep -E "rwkvtts manager|passed|failed" $O/m.log | head -12
done
