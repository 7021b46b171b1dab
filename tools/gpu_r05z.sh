set -o pipefail
mkdir -p gpurun_out/r05z
timeout -k 10 200 python3 -u tools/advance_stamps.py 64 > gpurun_out/r05z/adv.txt 2>&1; cat gpurun_out/r05z/adv.txt
