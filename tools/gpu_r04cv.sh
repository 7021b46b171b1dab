# k_conv with a scalar wave index (staging-issue branches on SGPRs) vs the previous library
# (build/abase): vocoder alone, alternating.
set -o pipefail
O=gpurun_out/r04cv
mkdir -p $O
B=RWKVTTS_LIB=$PWD/build/abase/librwkvtts.so
bash tools/codec_ab.sh X=1 "$B" X=1 "$B" > $O/codec_ab.txt 2>&1 || exit 1
grep -E "==|ms/batch|conv7|conv1|convT|total" $O/codec_ab.txt
