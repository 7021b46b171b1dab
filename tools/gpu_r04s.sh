# smoke(), then the bench (3 steps, with the B=1 leg) with in-graph kernel timing on / off,
# alternating, same box.
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
for a in "" "--no-graph-timing" "" "--no-graph-timing"; do
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline $a > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/b.json'))
print('[$a]', 'value', d['value'], 'decode_ms', d['decode_step_roofline']['ms_per_decode_step'], 'b1_us', d['batch1']['decode_step_us'], 'b1_sps', d['batch1']['samples_per_s'], 'dom', d['roofline']['kernel'], d['roofline']['avg_us'])" | tee -a $O/graph_timing_ab.txt
done
