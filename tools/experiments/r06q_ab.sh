# Round-6 A/B: the dilation-9 residual unit fused at 4 waves (17 staging blocks per wave) vs the
# round-6 head library: codec GPU tests, codec_bench with PCM digests, alternating.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06q_tests.txt 2>&1 || { tail -30 gpurun_out/r06q_tests.txt; exit 1; }
tail -2 gpurun_out/r06q_tests.txt
bash tools/codec_lib_ab.sh ab_libs/head/librwkvtts.so rwkv-tts-rs_amd/rwkvtts/librwkvtts.so 3 2>&1 | tee gpurun_out/r06q_codec_ab.txt
