# round 4: persistent FFN correctness + same-box decode A/B, then the new tests and a short bench
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ffn_persist.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/persist_tests.log 2>&1
rc=$?; echo "PERSIST TESTS EXIT $rc"; tail -8 $O/persist_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash tools/db_env_ab.sh 3 RWKVTTS_FFN_PERSIST=0 RWKVTTS_FFN_PERSIST=1 > $O/ab.txt 2>&1
rc=$?; echo "AB EXIT $rc"; cat $O/ab.txt; [ $rc -eq 0 ] || exit $rc
TAG=r04b/t PYTEST_ARGS="tests/test_gpu_advance.py tests/test_gpu_manager.py tests/test_gpu_fulllength.py tests/test_gpu_codec.py" bash tools/gpu_tests_then_bench.sh
