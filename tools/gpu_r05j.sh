set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
for b in 1 32; do
  RWKVTTS_LIB=$PWD/ab_libs/stl/librwkvtts.so timeout -k 10 120 python3 tools/ffn_stamps.py 32 ffn $b > $O/stl_b${b}_ffn.txt 2>&1 || exit 1
done
tail -n +1 $O/*.txt
