set -o pipefail
O=gpurun_out/r05ad
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_generate.py tests/test_gpu_batching.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; tail -3 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q -E "FAILED|ERROR" $O/tests.log || exit 1
timeout -k 10 200 python3 -u tools/advance_stamps.py 64 > $O/adv.txt 2>&1; tail -17 $O/adv.txt
T=rwkv-tts-rs_amd/rwkvtts/librwkvtts.so
TAG=r05ad BS="1 32" VARIANTS="ab_libs/head8/librwkvtts.so $T" STAMP_BS=none bash tools/gpu_r05_ab.sh
