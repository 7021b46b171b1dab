# Timeline (TL=1 build) of the decode step under RWKVTTS_DEBUG_EXP settings (timing only).
# Usage: bash tools/tl_exp.sh EXP...   (e.g. 0 1048576 2097152)
set -o pipefail
mkdir -p gpurun_out/tl
for e in "$@"; do
  echo "== RWKVTTS_DEBUG_EXP=$e"
  RWKVTTS_DEBUG_EXP=$e RWKVTTS_LIB=$PWD/build/tl/librwkvtts.so RWKVTTS_TIMELINE=$PWD/gpurun_out/tl/tl_x$e.txt timeout -k 10 120 python -u tools/decode_bench.py 64 1 | grep rep && python3 tools/timeline_summary.py gpurun_out/tl/tl_x$e.txt | grep -E "span|advance|gemm_head|embed" || exit 1
done
