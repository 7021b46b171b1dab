set -o pipefail
mkdir -p gpurun_out/r05q
RWKVTTS_LIB=$PWD/ab_libs/grandbg6/librwkvtts.so timeout -k 10 300 python3 -u tools/gran_debug.py > gpurun_out/r05q/debug.txt 2>&1; grep -c "GRANDBG " gpurun_out/r05q/debug.txt; grep GRANDBG6 gpurun_out/r05q/debug.txt | head -40; grep -v GRANDBG gpurun_out/r05q/debug.txt | tail -4
