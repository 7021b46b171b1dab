# Same-box decode A/B of environment settings, alternating N times (decode_bench S=512).
# Usage: db_env_ab.sh N ENV_A ENV_B
set -o pipefail
N=$1; shift
for r in $(seq 1 $N); do
  for e in "$@"; do
    echo -n "$e: "; env $e timeout -k 10 120 python -u tools/decode_bench.py 512 1 | grep -oE "decode [0-9.]+ us/step.*tokens [0-9a-f]+" | sed 's/ over.*tokens/ tokens/' || exit 1
  done
done
