# MFMA-busy counter pass: SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE per dispatch
# on the vocoder batch (codec_bench.py 32 x 512) and the LM decode (lm_short.py, eager), then a
# kernel-trace pass of the same commands for durations. Output under gpurun_out/mfma/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=${MFMA_OUT:-$R/gpurun_out/mfma}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export LM_GRAPHS=0
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES --output-format csv -d $O/codec_pmc -o run -- python3 $R/tools/codec_bench.py 32 512 > $O/codec_pmc.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/codec_kt -o run -- python3 $R/tools/codec_bench.py 32 512 > $O/codec_kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES --output-format csv -d $O/lm_pmc -o run -- python3 $R/tools/lm_short.py > $O/lm_pmc.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lm_kt -o run -- python3 $R/tools/lm_short.py > $O/lm_kt.log 2>&1
rc=$?; echo "MFMA PMC EXIT $rc"
python3 $R/tools/mfma_summary.py $O/codec_pmc $O/codec_kt > $O/codec_summary.txt 2>&1
python3 $R/tools/mfma_summary.py $O/lm_pmc $O/lm_kt > $O/lm_summary.txt 2>&1
cat $O/codec_summary.txt $O/lm_summary.txt
exit $rc
