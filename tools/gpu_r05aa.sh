set -o pipefail
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 300 python3 -u tools/gran_debug.py > $O/debug.txt 2>&1; tail -2 $O/debug.txt
grep -q "graphs False equal: True" $O/debug.txt || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_ffn_persist.py tests/test_gpu_generate.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; tail -3 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q -E "FAILED|ERROR" $O/tests.log || exit 1
T=rwkv-tts-rs_amd/rwkvtts/librwkvtts.so
TAG=r05aa BS="1" VARIANTS="ab_libs/head8/librwkvtts.so $T $T:RWKVTTS_RKV_GRAN=0" STAMP_BS=1 bash tools/gpu_r05_ab.sh
