# bench.py with several argument sets (short runs, no CPU baseline, no B=1 leg): value / ms_per_step /
# decode step / prefill. Usage: bash tools/bench_args_ab.sh "ARGS1" "ARGS2" ...   (ARGS may start with
# VAR=value environment assignments)
set -o pipefail
R=$GRAFT_REPO_ROOT
for e in "$@"; do
  env $(echo "$e" | tr ' ' '\n' | grep '=' | tr '\n' ' ') timeout -k 10 240 python3 $R/bench.py --steps ${BAB_STEPS:-3} --warmup 1 --no-cpu-baseline --no-batch1 $(echo "$e" | tr ' ' '\n' | grep -v '=' | tr '\n' ' ') > $R/gpurun_out/bab.json 2> $R/gpurun_out/bab.err || { tail -5 $R/gpurun_out/bab.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$R/gpurun_out/bab.json'))
print('$e |', 'value', d['value'], 'ms/step', d['ms_per_step'], 'decode_ms', d['decode_step_roofline']['ms_per_decode_step'], 'codec_ms', d['codec_roofline']['ms_per_batch'], 'breakdown', d['breakdown_ms_per_batch'])"
done
