set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batching.py tests/test_gpu_forward.py tests/test_gpu_generate.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_xmap.log 2>&1 || { tail -30 gpurun_out/t_xmap.log; exit 1; }
tail -2 gpurun_out/t_xmap.log
timeout -k 10 120 python -u tools/decode_bench.py 64 2 && RWKVTTS_NO_XMAP=1 timeout -k 10 120 python -u tools/decode_bench.py 64 2
