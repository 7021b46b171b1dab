set -o pipefail
A="RWKVTTS_LIB=$PWD/ab_libs/resv0/librwkvtts.so --no-graph-timing"
B="RWKVTTS_LIB=$PWD/ab_libs/resv1/librwkvtts.so --no-graph-timing"
C="--no-graph-timing"
D="RWKVTTS_LIB=$PWD/ab_libs/resv3/librwkvtts.so --no-graph-timing"
E="RWKVTTS_LIB=$PWD/ab_libs/resv4/librwkvtts.so --no-graph-timing"
for r in 1 2; do bash tools/bench_args_ab.sh "$A" "$B" "$C" "$D" "$E" || exit 1; done > gpurun_out/r06e_resv_ab.txt 2>&1
cat gpurun_out/r06e_resv_ab.txt
LIBS="ab_libs/r05/librwkvtts.so ab_libs/granv/librwkvtts.so rwkv-tts-rs_amd/rwkvtts/librwkvtts.so" BS="1" N=3 bash tools/db_multi_ab.sh > gpurun_out/r06e_gran_ab.txt 2>&1; cat gpurun_out/r06e_gran_ab.txt
