set -o pipefail
for e in 0 256 512 768; do
  echo "== exp $e"
  RWKVTTS_DEBUG_EXP=$e bash tools/prof_decode.sh e$e 32 | grep -E "steps=|gemm|ln_mix|wkv" || exit 1
done
