# A/B decode timing: each library in build/ab/*.so plus the in-tree build, same workload.
# Usage (GPU box): bash tools/ab.sh [S] [reps]
set -o pipefail
mkdir -p gpurun_out
S=${1:-64}; REPS=${2:-2}
for lib in build/ab/*.so rwkv-tts-rs_amd/rwkvtts/librwkvtts.so; do
  echo "== $lib"
  RWKVTTS_LIB=$PWD/$lib timeout -k 10 300 python -u tools/decode_bench.py $S $REPS || exit $?
done
