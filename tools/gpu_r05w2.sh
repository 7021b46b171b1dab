set -o pipefail
T=rwkv-tts-rs_amd/rwkvtts/librwkvtts.so
TAG=r05w2 BS="1" VARIANTS="$T:RWKVTTS_LAYER1=0 $T:RWKVTTS_L1_KHOLD=0 $T:RWKVTTS_L1_KHOLD=400 $T:RWKVTTS_L1_KHOLD=700 $T:RWKVTTS_L1_KHOLD=1000" STAMP_BS=none bash tools/gpu_r05_ab.sh
