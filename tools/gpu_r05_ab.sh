# Round-5 decode A/B: same-box decode_bench (S=256) at B=1 and B=32 over VARIANTS (each "LIB[:ENV...]":
# a library path, optionally followed by environment settings), alternating, 2 reps; then the
# persistent-launch stamps of the working tree (STAMP_ENV applied). TESTS=1 first runs the persistent
# bitwise / recovery suites.
set -o pipefail
O=gpurun_out/${TAG:-r05a}
mkdir -p $O
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_ffn_persist.py tests/test_gpu_persist_recovery.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; tail -12 $O/tests.log
  grep -q " passed" $O/tests.log && ! grep -q -E "FAILED|ERROR" $O/tests.log || exit 1
fi
for r in 1 2; do for b in ${BS:-1 32}; do for V in $VARIANTS; do
  L=${V%%:*}; E=""; [ "$V" != "$L" ] && E=${V#*:}; E=${E//:/ }
  echo -n "B=$b $V: "; env $E RWKVTTS_LIB=$PWD/$L DB_B=$b timeout -k 10 120 python -u tools/decode_bench.py 256 1 | grep -oE "decode [0-9.]+ us/step.*tokens [0-9a-f]+" || exit 1
done; done; done > $O/ab.txt 2>&1
cat $O/ab.txt
[ "${STAMP_BS:-}" = none ] && exit 0
for w in att ffn; do for b in ${STAMP_BS:-1 32}; do
  env $STAMP_ENV timeout -k 10 120 python3 tools/ffn_stamps.py 32 $w $b > $O/stamps_b${b}_$w.txt 2>&1 || exit 1
done; done
tail -n +1 $O/stamps_*.txt
