# B = 1 decode step vs the split-K of its GEMMs (env; decode_bench DB_B=1, separate launches).
set -o pipefail
O=gpurun_out/r04b1b
mkdir -p $O
for r in 1 2; do
for e in "X=1" "RWKVTTS_RKV_KS=512" "RWKVTTS_KEY_KS=512" "RWKVTTS_VAL_KS=512" "RWKVTTS_WO_KS=256" "RWKVTTS_HEAD_KS=1024"; do
  echo -n "$e: "; env $e DB_B=1 timeout -k 10 120 python -u tools/decode_bench.py 256 1 | grep -oE "decode [0-9.]+ us/step.*tokens [0-9a-f]+" | sed 's/ over.*tokens/ tokens/' || exit 1
done
done > $O/ab.txt 2>&1
cat $O/ab.txt
