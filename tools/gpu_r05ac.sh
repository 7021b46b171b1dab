set -o pipefail
mkdir -p gpurun_out/r05ac
timeout -k 10 200 python3 -u tools/advance_stamps.py 64 > gpurun_out/r05ac/adv.txt 2>&1; tail -18 gpurun_out/r05ac/adv.txt
