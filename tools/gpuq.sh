#!/bin/bash
# usage: gpuq.sh <logfile> <timeout> <cmd>; retries only while no GPU slot is free (exit 3)
log=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "rc=$rc" >> $log; exit $rc; fi
  sleep 90
done
echo "gave up (no slot)" >> $log
