# Prefill-only A/B (tools/prefill_trace.py): 128-row GEMM groups, relu^2 planes, chunk 512 / 2048
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_batching.py tests/test_gpu_generate.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pf_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/pf_tests.log; exit 1; }
tail -1 gpurun_out/pf_tests.log
for c in 512 2048; do
  for v in "RWKVTTS_NO_BIG_MT=1 RWKVTTS_NO_RELU2_PLANES=1" "RWKVTTS_NO_BIG_MT=1" "RWKVTTS_NO_RELU2_PLANES=1" "X=1"; do
    r=$(env $v PF_CHUNK=$c timeout -k 10 120 python tools/prefill_trace.py | tail -1) || exit 1
    echo "chunk=$c $v: $r"
  done
done
