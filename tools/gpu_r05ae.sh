set -o pipefail
O=gpurun_out/r05ae
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_persist_recovery.py tests/test_gpu_sampler.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; tail -8 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q -E "FAILED|ERROR" $O/tests.log || exit 1
