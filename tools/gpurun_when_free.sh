# Run one gpurun call, re-submitting it only while the pool has no box for it (nothing ran and
# nothing was charged: "no free box", "slots busy", "backing off"); stops at the first call that ran
# (whatever its result). Usage: gpurun_when_free.sh LOG TIMEOUT 'command'
LOG=$1; TMO=$2; CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $TMO -- "$CMD" > $LOG 2>&1
  if grep -qE "no free box|slot\(s\) on this pod are busy|backing off|another call|stopped responding while being prepared" $LOG && ! grep -q "charged=[1-9]" $LOG; then
    w=$(grep -oE "retry in [0-9]+s" $LOG | grep -oE "[0-9]+" | head -1); sleep ${w:-90}; sleep 30
    continue
  fi
  break
done
