set -o pipefail
timeout -k 10 600 python -m pytest tests/test_gpu_forward.py tests/test_gpu_generate.py -x -q > gpurun_out/fwd.log 2>&1; rc=$?
echo "TESTS $rc"; tail -3 gpurun_out/fwd.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/wkv_rows.py && RWKVTTS_DEBUG_EXP=0 timeout -k 10 120 python tools/wkv_stamps.py
