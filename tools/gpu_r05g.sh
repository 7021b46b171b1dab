set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
for w in ffn att; do for b in 32 1; do
  RWKVTTS_LIB=$PWD/ab_libs/stx/librwkvtts.so timeout -k 10 120 python3 tools/ffn_stamps.py 32 $w $b > $O/stx_b${b}_$w.txt 2>&1 || exit 1
done; done
tail -n +1 $O/*.txt
