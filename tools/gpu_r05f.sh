set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_ffn_persist.py tests/test_gpu_persist_recovery.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; tail -12 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q -E "FAILED|ERROR" $O/tests.log || exit 1
TAG=r05f BS="32 1" VARIANTS="ab_libs/base/librwkvtts.so ab_libs/fused1/librwkvtts.so rwkv-tts-rs_amd/rwkvtts/librwkvtts.so" STAMP_BS=1 bash tools/gpu_r05_ab.sh
