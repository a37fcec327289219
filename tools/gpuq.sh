#!/bin/bash
# usage: gpuq.sh LOG TIMEOUT CMD -- retries only while gpurun reports no free box (rc 3)
log=$1; to=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "no free box\|backing off\|busy" $log; then break; fi
  sleep 120
done
echo "rc=$rc tries=$i" >> $log
