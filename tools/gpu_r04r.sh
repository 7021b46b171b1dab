# Round-4 bench of record (10 steps, CPU baseline, B=1 leg) + rocprof profiles, then pipelining /
# vocoder-tile A/Bs of the bench.
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 10 --warmup 1 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
bash tools/gpu_profiles.sh r04c || exit 1
bash tools/bench_args_ab.sh "" "--voc-delay-ms 12" "RWKVTTS_CONV7_TN=96" "RWKVTTS_CODEC_CUS=128" "" > $O/bench_ab.txt 2>&1
cat $O/bench_ab.txt
timeout -k 10 120 python3 tools/ffn_stamps.py 32 att 1 > $O/stamps_b1_att.txt 2>&1 && \
timeout -k 10 120 python3 tools/ffn_stamps.py 32 ffn 1 > $O/stamps_b1_ffn.txt 2>&1 && \
timeout -k 10 120 python3 tools/ffn_stamps.py 32 att 32 > $O/stamps_b32_att.txt 2>&1
cat $O/stamps_*.txt
