set -o pipefail
mkdir -p gpurun_out/r05n
timeout -k 10 300 python3 -u tools/gran_debug.py > gpurun_out/r05n/debug.txt 2>&1; cat gpurun_out/r05n/debug.txt | tail -20
