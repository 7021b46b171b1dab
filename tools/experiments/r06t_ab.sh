# Round-6 A/B: 192-channel pointwise convs 64-wide (ab_libs/pw64) vs the final tree: PCM digest, bench x3 alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
bash tools/codec_lib_ab.sh rwkv-tts-rs_amd/rwkvtts/librwkvtts.so ab_libs/pw64/librwkvtts.so 1 2>&1 | grep -E "==|digest|ms/batch|res_conv1@192|total" | tee gpurun_out/r06t_codec.txt || exit 1
for r in 1 2 3; do
bash tools/bench_ab.sh RWKVTTS_X=1 RWKVTTS_LIB=$R/ab_libs/pw64/librwkvtts.so 2>&1 | tee -a gpurun_out/r06t_bab.txt || exit 1
done
