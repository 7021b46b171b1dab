# Prefill-only workload (the bench's 32 prompts in one 1280-row step) under RWKVTTS_GEMM_RPW
# settings (row groups per GEMM workgroup; 0 = the launcher's default). Usage: prefill_rpw_ab.sh RPW...
set -o pipefail
for rpw in "$@"; do
echo "== RWKVTTS_GEMM_RPW=$rpw"; RWKVTTS_GEMM_RPW=$rpw PF_CHUNK=2048 timeout -k 10 120 python3 tools/prefill_trace.py | tail -1 || exit 1
done
