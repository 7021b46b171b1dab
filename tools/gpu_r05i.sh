set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ffn_persist.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; tail -5 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q -E "FAILED|ERROR" $O/tests.log || exit 1
TAG=r05i BS="32 1" VARIANTS="ab_libs/base/librwkvtts.so ab_libs/hd_xmin/librwkvtts.so rwkv-tts-rs_amd/rwkvtts/librwkvtts.so" STAMP_BS=none bash tools/gpu_r05_ab.sh
