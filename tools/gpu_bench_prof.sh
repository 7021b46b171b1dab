set -o pipefail
mkdir -p gpurun_out/r01_v1
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/r01_v1/bench.json 2> gpurun_out/r01_v1/bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r01_v1/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r01_v1/prof.log 2>&1
echo EXIT $?
