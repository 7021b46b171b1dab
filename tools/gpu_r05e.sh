set -o pipefail
TAG=r05e BS="32 1" VARIANTS="ab_libs/base/librwkvtts.so rwkv-tts-rs_amd/rwkvtts/librwkvtts.so ab_libs/xmin/librwkvtts.so ab_libs/pad/librwkvtts.so ab_libs/att3/librwkvtts.so ab_libs/wpc3/librwkvtts.so" STAMP_BS=none bash tools/gpu_r05_ab.sh
