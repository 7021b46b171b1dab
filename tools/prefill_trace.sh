set -o pipefail
# kernel trace of a short decode_bench run: the first steps are the 512-row prefill steps
export TMPDIR=/tmp
mkdir -p gpurun_out/pf
env "$@" timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pf -o pf -- python3 tools/decode_bench.py 4 1 && \
python3 tools/trace_steps.py gpurun_out/pf 5
