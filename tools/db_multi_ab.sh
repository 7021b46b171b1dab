# Same-box decode A/B over several library builds, alternating (tools/decode_bench.py, graph replay):
# µs per step and the token checksum of every run (a change that keeps the arithmetic keeps it).
# Usage: LIBS="ab_libs/a/librwkvtts.so rwkv-tts-rs_amd/rwkvtts/librwkvtts.so" [BS="1 32"] [N=3] [S=256] bash tools/db_multi_ab.sh
set -o pipefail
for r in $(seq 1 ${N:-3}); do for b in ${BS:-32}; do for L in $LIBS; do
  echo -n "B=$b $L: "
  DB_B=$b RWKVTTS_LIB=$PWD/$L timeout -k 10 120 python -u tools/decode_bench.py ${S:-256} 1 | grep -oE "decode [0-9.]+ us/step.*tokens [0-9a-f]+" || exit 1
done; done; done
