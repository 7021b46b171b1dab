# k_advance duration in the TL=1 launch timeline: normal prompts (32 global + S semantic steps)
# vs zero-shot prompts (semantic steps only). Usage: bash tools/tl_adv.sh S
set -o pipefail
mkdir -p gpurun_out/tl
for zs in 0 1; do
  echo "== DB_ZS=$zs S=$1"
  DB_ZS=$zs RWKVTTS_LIB=$PWD/build/tl/librwkvtts.so RWKVTTS_DEBUG_STAMPS=timeline=$PWD/gpurun_out/tl/tl_zs$zs.txt timeout -k 10 120 python -u tools/decode_bench.py $1 1 | grep rep && python3 tools/timeline_summary.py gpurun_out/tl/tl_zs$zs.txt | grep -E "span|advance|gemm_head" || exit 1
done
