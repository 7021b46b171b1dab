set -o pipefail
echo "== default"; timeout -k 10 120 python -u tools/decode_bench.py 64 2 | tail -1 || exit 1
echo "== HIP_FORCE_DEV_KERNARG=1"; HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python -u tools/decode_bench.py 64 2 | tail -1 || exit 1
echo "== HIP_FORCE_DEV_KERNARG=0"; HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 python -u tools/decode_bench.py 64 2 | tail -1 || exit 1
