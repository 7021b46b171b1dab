# Same-box A/B of the window-end wait (RWKVTTS_SYNC_BLOCKING): bench without CPU baseline
set -o pipefail
for e in RWKVTTS_SYNC_BLOCKING=1 X=0 RWKVTTS_SYNC_BLOCKING=1 X=0; do
  env $e timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/sy.json 2>gpurun_out/sy.err || exit 1
  python3 -c "
import json;d=json.loads(open('gpurun_out/sy.json').read().strip().splitlines()[-1]);b=d['breakdown_ms_per_batch'];print('$e', d['value'], b, round(b['generate']-b['decode']-b['prefill'],2))"
done
