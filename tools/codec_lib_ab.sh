# Same-box vocoder A/B of two library builds, alternating N times: codec_bench 32 x 512 per build,
# with a digest of the PCM (bitwise comparison). Usage: codec_lib_ab.sh LIB_A LIB_B N
set -o pipefail
for r in $(seq 1 ${3:-3}); do
  for L in "$1" "$2"; do
    echo "== $L"; CODEC_DIGEST=1 RWKVTTS_LIB=$PWD/$L timeout -k 10 120 python -u tools/codec_bench.py 32 512 || exit 1
  done
done
