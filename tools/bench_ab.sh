# bench.py under several environment settings (short runs, no CPU baseline): value / ms_per_step /
# decode step. Usage: bash tools/bench_ab.sh ENV...
set -o pipefail
R=$GRAFT_REPO_ROOT
for e in "$@"; do
  env $e timeout -k 10 200 python3 $R/bench.py --steps ${BAB_STEPS:-3} --warmup 1 --no-cpu-baseline > $R/gpurun_out/bab.json 2> $R/gpurun_out/bab.err || { tail -5 $R/gpurun_out/bab.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$R/gpurun_out/bab.json'))
print('$e', 'value', d['value'], 'ms/step', d['ms_per_step'], 'decode_ms', d['decode_step_roofline']['ms_per_decode_step'], 'codec_ms', d['codec_roofline']['ms_per_batch'], 'att_us', round(d['kernels'].get('att_persist',{}).get('avg_us',0),2), 'b1_us', d.get('batch1',{}).get('decode_step_us'))"
done
