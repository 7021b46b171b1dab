set -o pipefail
for e in 0 524288; do
  echo "== exp $e"
  RWKVTTS_DEBUG_EXP=$e timeout -k 10 120 python -u tools/decode_bench.py 64 2 | tail -1 || exit 1
  RWKVTTS_DEBUG_EXP=$e bash tools/prof_decode.sh x$e 32 | grep -E "gemm<2, 8, 0, false> g13|wkv" || exit 1
done
