set -o pipefail
mkdir -p gpurun_out/emb
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/emb/tests.log 2>&1 || { tail -30 gpurun_out/emb/tests.log; exit 1; }
tail -1 gpurun_out/emb/tests.log
bash tools/lib_ab.sh build_ab/head2_tl/librwkvtts.so build/tl/librwkvtts.so build_ab/head2/librwkvtts.so rwkv-tts-rs_amd/rwkvtts/librwkvtts.so 2>&1 | grep -E "==|rep|span|embed|ln_att"
