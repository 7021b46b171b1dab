# Same-box A/B of two library builds: TL=1 launch timelines (decode_bench S=256, semantic steps)
# and graph-replayed decode step times. Usage: lib_ab.sh TL_LIB_A TL_LIB_B LIB_A LIB_B
set -o pipefail
mkdir -p gpurun_out/ab
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then L=$1; P=$3; else L=$2; P=$4; fi
    echo "== $v"
    RWKVTTS_LIB=$PWD/$L RWKVTTS_DEBUG_STAMPS=timeline=$PWD/gpurun_out/ab/tl_$v.txt timeout -k 10 120 python -u tools/decode_bench.py 256 1 | grep rep && python3 tools/timeline_summary.py gpurun_out/ab/tl_$v.txt || exit 1
    RWKVTTS_LIB=$PWD/$P timeout -k 10 120 python -u tools/decode_bench.py 256 2 | grep rep || exit 1
  done
done
