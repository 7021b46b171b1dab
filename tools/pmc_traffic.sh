# HBM traffic per kernel: two separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE), eager launches.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
export LM_GRAPHS=0
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc/fetch -o run -- python3 $R/tools/lm_short.py > $R/gpurun_out/pmc/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc/write -o run -- python3 $R/tools/lm_short.py > $R/gpurun_out/pmc/write.log 2>&1
rc=$?; echo "PMC EXIT $rc"; find $R/gpurun_out/pmc -name "*.csv" | head; exit $rc
