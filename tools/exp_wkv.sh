set -o pipefail
for e in 0 1 2 4 7; do
  RWKVTTS_DEBUG_EXP=$e timeout -k 10 120 python tools/wkv_stamps.py > gpurun_out/exp_$e.log 2>&1 || exit 1
  echo "== exp $e"; cat gpurun_out/exp_$e.log
done
