# Sampler change check on the GPU: sampler / generate / batching / full-length parity tests, then
# the TL=1 launch timeline of the decode step (k_advance mean over semantic steps) against a
# reference TL build ($1), then eager per-kernel times (advance_ab.py) against a reference build ($2).
set -o pipefail
mkdir -p gpurun_out/samp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_generate.py tests/test_gpu_batching.py tests/test_gpu_fulllength.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/samp/tests.log 2>&1 || { tail -30 gpurun_out/samp/tests.log; exit 1; }
tail -2 gpurun_out/samp/tests.log
for r in 1 2; do
  for v in ref new; do
    if [ $v = ref ]; then L=$PWD/$1; else L=$PWD/build/tl/librwkvtts.so; fi
    echo "== $v"
    RWKVTTS_LIB=$L RWKVTTS_DEBUG_STAMPS=timeline=$PWD/gpurun_out/samp/tl_$v.txt timeout -k 10 120 python -u tools/decode_bench.py 256 1 | grep rep && python3 tools/timeline_summary.py gpurun_out/samp/tl_$v.txt | grep -E "span|advance|head" || exit 1
  done
done
for lib in "$2" ""; do
  echo "== eager lib=${lib:-new}"
  RWKVTTS_LIB=$lib timeout -k 10 120 python3 tools/advance_ab.py 256 2>&1 | grep sample_advance || exit 1
done
