set -o pipefail
timeout -k 10 600 python -m pytest tests/test_gpu_sampler.py tests/test_gpu_generate.py -x -q > gpurun_out/samp.log 2>&1; rc=$?
echo "TESTS $rc"; tail -3 gpurun_out/samp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sampler_stamps.py
