# Sampler change check on the GPU: sampler / generate / batching / full-length parity tests, then
# k_advance phase stamps, then a same-box decode A/B against a reference build (RWKVTTS_LIB=$1).
set -o pipefail
mkdir -p gpurun_out/samp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_generate.py tests/test_gpu_batching.py tests/test_gpu_fulllength.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/samp/tests.log 2>&1 || { tail -30 gpurun_out/samp/tests.log; exit 1; }
tail -2 gpurun_out/samp/tests.log
timeout -k 10 180 python tools/advance_stamps.py 64 > gpurun_out/samp/stamps.txt 2>&1 || exit 1
cat gpurun_out/samp/stamps.txt
for r in 1 2; do
  for lib in "$1" ""; do
    echo "== lib=${lib:-new}"
    RWKVTTS_LIB=$lib timeout -k 10 120 python3 tools/decode_bench.py 256 2 2>&1 | grep "rep " || exit 1
    RWKVTTS_LIB=$lib timeout -k 10 120 python3 tools/advance_ab.py 64 2>&1 | grep sample_advance || exit 1
  done
done
