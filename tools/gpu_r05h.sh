set -o pipefail
TAG=r05h BS="32" VARIANTS="ab_libs/base/librwkvtts.so ab_libs/r4/librwkvtts.so ab_libs/af_xmin/librwkvtts.so ab_libs/hd_xmin/librwkvtts.so ab_libs/xmin/librwkvtts.so rwkv-tts-rs_amd/rwkvtts/librwkvtts.so ab_libs/codepad/librwkvtts.so" STAMP_BS=none bash tools/gpu_r05_ab.sh
