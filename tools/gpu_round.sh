# One GPU session (one gpurun call): the -m gpu suite (full-length report kept), smoke, bench.py's
# default line, the rocprof kernel-trace + PMC traffic profiles of the bench (gpu_profiles.sh) and the
# MFMA-busy counter passes (pmc_mfma.sh), any subset, each step under its own time limit; the first
# failing step ends the call. Every summary is stamped with the library's build id
# (rwkvtts._ffi.build_id()), which bench.py matches when it cites profiles/.
# Usage: bash tools/gpu_round.sh TAG [STEPS]   STEPS: comma list of suite,smoke,bench,prof,mfma (default all)
# Outputs: gpurun_out/TAG/ (suite, smoke, bench line), gpurun_out/prof_TAG/, gpurun_out/mfma_TAG/;
# then on the CPU side: bash tools/keep_profiles.sh TAG copies the summaries into profiles/.
set -o pipefail
T=${1:?usage: gpu_round.sh TAG [STEPS]}
S=${2:-suite,smoke,bench,prof,mfma}
O=gpurun_out/$T
mkdir -p $O
has() { [[ ",$S," == *",$1,"* ]]; }
python3 -c "import sys; sys.path.insert(0, 'rwkv-tts-rs_amd'); from rwkvtts import _ffi; print(_ffi.build_id())" > $O/build_id.txt
echo "build $(cat $O/build_id.txt)"
if has suite; then
  RWKVTTS_REPORT_DIR=$PWD/$O timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_suite.txt; exit 1; }
  tail -2 $O/gpu_suite.txt
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKE FAILED; tail $O/smoke.txt; exit 1; }
  tail -1 $O/smoke.txt
fi
if has bench; then
  timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
  tail -c 300 $O/bench.json
fi
if has prof; then
  bash tools/gpu_profiles.sh $T || { echo PROFILES FAILED; exit 1; }
fi
if has mfma; then
  MFMA_OUT=$PWD/gpurun_out/mfma_$T bash tools/pmc_mfma.sh || { echo MFMA FAILED; exit 1; }
fi
echo ROUND_OK
