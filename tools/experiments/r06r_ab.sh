# Round-6 A/B: the vocoder's activation streams non-temporal (ab_libs/cnt) vs the tree: PCM digest,
# then bench.py --steps 3 alternating x3 (decode step beside the vocoder).
set -o pipefail
R=$GRAFT_REPO_ROOT
bash tools/codec_lib_ab.sh rwkv-tts-rs_amd/rwkvtts/librwkvtts.so ab_libs/cnt/librwkvtts.so 1 2>&1 | grep -E "==|digest|ms/batch|total" | tee gpurun_out/r06r_codec.txt || exit 1
for r in 1 2 3; do
bash tools/bench_ab.sh RWKVTTS_X=1 RWKVTTS_LIB=$R/ab_libs/cnt/librwkvtts.so 2>&1 | tee -a gpurun_out/r06r_bab.txt || exit 1
done
