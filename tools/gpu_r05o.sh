set -o pipefail
mkdir -p gpurun_out/r05o
RWKVTTS_LIB=$PWD/ab_libs/grandbg2/librwkvtts.so timeout -k 10 300 python3 -u tools/gran_debug.py > gpurun_out/r05o/debug.txt 2>&1; grep -c GRANDBG2 gpurun_out/r05o/debug.txt; grep GRANDBG2 gpurun_out/r05o/debug.txt | head -30; grep -v GRANDBG2 gpurun_out/r05o/debug.txt | tail
