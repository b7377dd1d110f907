#!/bin/bash
# usage: gpurun_retry.sh LOG SCRIPT [timeout]  -- retries only while gpurun reports no free slot (rc 3)
LOG=$1; SCRIPT=$2; TO=${3:-1200}
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $TO -- bash $SCRIPT > $LOG 2>&1; rc=$?
  if [ $rc -ne 3 ] && ! grep -q "slot(s) on this pod are busy" $LOG; then break; fi
  sleep 150
done
echo "done rc=$rc" >> $LOG
