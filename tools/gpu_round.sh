set -o pipefail
mkdir -p gpurun_out/${TAG:-r02c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r02c}/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${TAG:-r02c}/gpu_tests.log; exit 1; }
tail -2 gpurun_out/${TAG:-r02c}/gpu_tests.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG:-r02c}/bench.json 2> gpurun_out/${TAG:-r02c}/bench.err || { echo BENCH FAILED; tail gpurun_out/${TAG:-r02c}/bench.err; exit 1; }
tail -c 600 gpurun_out/${TAG:-r02c}/bench.json
bash tools/gpu_profiles.sh ${TAG:-r02c}
