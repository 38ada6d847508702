#!/bin/bash
# usage: bash scripts/gpurun_retry.sh LOGFILE <gpurun args...>  (retries only "no box" outcomes)
# retry gpurun only while no box could be acquired (nothing ran, nothing charged)
LOG=$1; shift
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun "$@" > $LOG 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "no free box right now\|stopped responding while being prepared\|backing off\|GPU slot(s) on this pod are busy\|status=transient" $LOG; then
    if grep -q "status=ok" $LOG; then break; fi
    sleep 90
    continue
  fi
  break
done
echo "done rc=$rc tries=$i" >> $LOG
