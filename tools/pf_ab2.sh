set -o pipefail
for cfg in "0 8 0" "1 8 0" "1 2 0" "1 8 1"; do
  set -- $cfg
  RWKVTTS_PREFETCH=$1 RWKVTTS_PREFETCH_BLOCKS=$2 RWKVTTS_PREFETCH_STATE=$3 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pfb.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/pfb.json').read().strip().splitlines()[-1])
print('cfg $cfg', d['value'], d['ms_per_step'], d['decode_step_roofline']['ms_per_decode_step'])"
done
