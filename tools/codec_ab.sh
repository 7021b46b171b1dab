# codec_bench.py (32 x 512) under several environment settings. Usage: bash tools/codec_ab.sh ENV...
set -o pipefail
R=$GRAFT_REPO_ROOT
for e in "$@"; do
  echo "== $e"
  env $e timeout -k 10 120 python3 $R/tools/codec_bench.py 32 512 2>&1 || exit 1
done
