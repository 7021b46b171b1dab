set -o pipefail
# needs the TL=1 build: make -C rwkv-tts-rs_amd/csrc TL=1
mkdir -p gpurun_out
for e in "$@"; do
echo "== $e"
env $e RWKVTTS_LIB=$PWD/build/tl/librwkvtts.so RWKVTTS_DEBUG_STAMPS=timeline=$PWD/gpurun_out/timeline.txt timeout -k 10 120 python -u tools/decode_bench.py 64 1 && python3 tools/timeline_summary.py gpurun_out/timeline.txt || exit 1
done
