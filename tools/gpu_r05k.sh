set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ffn_persist.py tests/test_gpu_batching.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; tail -3 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q -E "FAILED|ERROR" $O/tests.log || exit 1
T=rwkv-tts-rs_amd/rwkvtts/librwkvtts.so
TAG=r05k BS="1" VARIANTS="ab_libs/head3/librwkvtts.so $T $T:RWKVTTS_PF_HOLD=100,0,0,150,100 $T:RWKVTTS_PF_HOLD=100,0,0,300,100 $T:RWKVTTS_PF_HOLD=100,300,0,0,100 $T:RWKVTTS_PF_HOLD=100,300,0,300,100" STAMP_BS=none bash tools/gpu_r05_ab.sh || exit 1
TAG=r05k2 BS="32" VARIANTS="ab_libs/head3/librwkvtts.so $T" STAMP_BS=none bash tools/gpu_r05_ab.sh
