# Same-box A/B of the host-side window handling (env switches given as arguments): bench without
# CPU baseline, per-batch breakdown and the host time outside the GPU units
set -o pipefail
for e in "$@"; do
  env $e timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/sy.json 2>gpurun_out/sy.err || exit 1
  python3 -c "
import json;d=json.loads(open('gpurun_out/sy.json').read().strip().splitlines()[-1]);b=d['breakdown_ms_per_batch'];print('$e', d['value'], b, round(b['generate']-b['decode']-b['prefill'],2))"
done
