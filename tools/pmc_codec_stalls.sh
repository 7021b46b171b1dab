# Stall breakdown of the vocoder kernels (codec_bench.py 32 x 512): two counter passes, summarised
# per kernel class by tools/pmc_stalls_summary.py. Output under gpurun_out/stalls/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/stalls
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/a -o run -- python3 $R/tools/codec_bench.py 32 512 > $O/a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_DATA_FIFO_FULL SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/b -o run -- python3 $R/tools/codec_bench.py 32 512 > $O/b.log 2>&1
rc=$?; echo "STALL PMC EXIT $rc"
python3 $R/tools/pmc_stalls_summary.py $O/a $O/b > $O/summary.txt 2>&1
cat $O/summary.txt
exit $rc
