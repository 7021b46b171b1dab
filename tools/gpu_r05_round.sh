# Round-5 GPU round: the whole -m gpu suite (full-length report kept), bench.py's default line,
# the rocprof kernel-trace + PMC traffic profiles, and the MFMA-busy counter passes.
# Usage: TAG=r05r bash tools/gpu_r05_round.sh
set -o pipefail
T=${TAG:-r05r}
O=gpurun_out/$T
mkdir -p $O
RWKVTTS_REPORT_DIR=$PWD/$O timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKE FAILED; tail $O/smoke.txt; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
tail -c 300 $O/bench.json
bash tools/gpu_profiles.sh $T || exit 1
[ "${MFMA:-1}" = 1 ] && { bash tools/pmc_mfma.sh || exit 1; }
echo ROUND_OK
