set -o pipefail
timeout -k 10 600 python -m pytest tests/test_gpu_forward.py tests/test_gpu_generate.py -x -q > gpurun_out/pf_tests.log 2>&1; rc=$?
echo "TESTS $rc"; tail -2 gpurun_out/pf_tests.log; [ $rc -eq 0 ] || exit $rc
for pf in 0 1; do
  RWKVTTS_PREFETCH=$pf timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pf_$pf.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/pf_$pf.json').read().strip().splitlines()[-1])
print('prefetch=$pf', d['value'], d['ms_per_step'], d['decode_step_roofline']['ms_per_decode_step'], {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})"
done
