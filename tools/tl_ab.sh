set -o pipefail
mkdir -p gpurun_out/tl
for r in 1 2; do
for v in head new; do
  if [ $v = head ]; then L=$PWD/build_ab/head_tl/librwkvtts.so; else L=$PWD/build/tl/librwkvtts.so; fi
  echo "== $v"
  RWKVTTS_LIB=$L RWKVTTS_DEBUG_STAMPS=timeline=$PWD/gpurun_out/tl/tl_$v.txt timeout -k 10 120 python -u tools/decode_bench.py 64 1 | grep rep && python3 tools/timeline_summary.py gpurun_out/tl/tl_$v.txt | tail -14 || exit 1
done
done
