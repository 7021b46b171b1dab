# A/B decode timing over env settings: bash tools/ab_env.sh S REPS "VAR=a" "VAR=b" ...
set -o pipefail
S=$1; REPS=$2; shift 2
for e in "$@"; do
  echo "== $e"
  env $e timeout -k 10 120 python -u tools/decode_bench.py $S $REPS | tail -1 || exit 1
done
