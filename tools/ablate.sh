set -o pipefail
for e in 0 768 65536 131072 262144 458752; do
  echo "== exp $e"
  RWKVTTS_DEBUG_EXP=$e timeout -k 10 120 python -u tools/decode_bench.py 64 2 | tail -1 || exit 1
done
