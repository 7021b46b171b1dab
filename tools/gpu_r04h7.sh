# Small batches: the persistent halves (RWKVTTS_PERSIST_MIN_ROWS=1) with the weight-stream hold vs
# the separate launches (default below 16 rows), B = 1 and 8.
set -o pipefail
O=gpurun_out/r04h7
mkdir -p $O
for r in 1 2; do
for b in 1 8; do
for e in "X=1" "RWKVTTS_PERSIST_MIN_ROWS=1" "RWKVTTS_PERSIST_MIN_ROWS=1 RWKVTTS_PF_HOLD=200,0,0,0,200" "RWKVTTS_PERSIST_MIN_ROWS=1 RWKVTTS_PF_HOLD=50,0,0,0,50"; do
  echo -n "B=$b $e: "; env $e DB_B=$b timeout -k 10 120 python -u tools/decode_bench.py 256 1 | grep -oE "decode [0-9.]+ us/step" || exit 1
done; done; done > $O/ab.txt 2>&1
cat $O/ab.txt
