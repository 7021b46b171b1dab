set -o pipefail
mkdir -p gpurun_out/r05p
for v in gv3; do echo "== $v"; RWKVTTS_LIB=$PWD/ab_libs/$v/librwkvtts.so timeout -k 10 300 python3 -u tools/gran_debug.py 2>&1 | tail -6; done
