# Pointwise conv column-tile width after the buffer-load staging: 96 (default) vs 192 vs 64.
set -o pipefail
O=gpurun_out/r04cx
mkdir -p $O
bash tools/codec_ab.sh X=1 RWKVTTS_CONV1_TN=192 RWKVTTS_CONV1_TN=64 X=1 RWKVTTS_CONV1_TN=192 > $O/codec_ab.txt 2>&1 || exit 1
grep -E "==|ms/batch|conv1|total" $O/codec_ab.txt
