set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
for r in 1 2; do for b in 1 32; do for L in build/rev/base/librwkvtts.so rwkv-tts-rs_amd/rwkvtts/librwkvtts.so; do
  echo -n "B=$b $L: "; RWKVTTS_LIB=$PWD/$L DB_B=$b timeout -k 10 120 python -u tools/decode_bench.py 256 1 | grep -oE "decode [0-9.]+ us/step.*tokens [0-9a-f]+" || exit 1
done; done; done > $O/ab.txt 2>&1
cat $O/ab.txt
timeout -k 10 120 python3 tools/ffn_stamps.py 32 att 1 > $O/stamps_b1_att.txt 2>&1 && \
timeout -k 10 120 python3 tools/ffn_stamps.py 32 ffn 1 > $O/stamps_b1_ffn.txt 2>&1 && \
timeout -k 10 120 python3 tools/ffn_stamps.py 32 att 32 > $O/stamps_b32_att.txt 2>&1 && \
timeout -k 10 120 python3 tools/ffn_stamps.py 32 ffn 32 > $O/stamps_b32_ffn.txt 2>&1
cat $O/stamps_*.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_persist_recovery.py -x -v --timeout 300 --timeout-method thread > $O/recovery.log 2>&1; tail -15 $O/recovery.log
