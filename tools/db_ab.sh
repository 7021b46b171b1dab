# decode_bench.py (S=256, 2 reps) under several environment settings; prints the rep lines.
# Usage: bash tools/db_ab.sh ENV...
set -o pipefail
R=$GRAFT_REPO_ROOT
for e in "$@"; do
  echo "== $e"
  env $e timeout -k 10 120 python3 $R/tools/decode_bench.py 256 2 2>&1 | grep "rep " || exit 1
done
