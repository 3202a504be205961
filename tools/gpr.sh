#!/bin/bash
# usage: gpr.sh <logfile> <timeout> '<command>'  -- retries only while the pool has no box (nothing ran)
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if grep -q "no free box right now\|backing off after the last attempt failed on the infrastructure side\|stopped responding while being prepared\|GPU slot(s) on this pod are busy" $LOG && ! grep -q "rc=[0-9]" $LOG; then
    sleep 90; continue
  fi
  echo "gpurun rc=$rc after $i attempts" >> $LOG
  exit $rc
done
