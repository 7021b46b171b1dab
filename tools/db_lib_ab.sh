# Same-box decode A/B of two library builds, alternating N times (decode_bench S=512, 1 rep each).
# Usage: db_lib_ab.sh LIB_A LIB_B N
set -o pipefail
for r in $(seq 1 ${3:-4}); do
  for L in "$1" "$2"; do
    echo -n "$L: "; RWKVTTS_LIB=$PWD/$L timeout -k 10 120 python -u tools/decode_bench.py 512 1 | grep -oE "decode [0-9.]+ us/step" || exit 1
  done
done
