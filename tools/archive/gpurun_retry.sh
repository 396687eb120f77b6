#!/bin/bash
# usage: tools/gpurun_retry.sh LOG [gpurun args...]
# gpurun with retries while the pool has no box (exit 3: nothing ran, nothing charged)
LOG=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@" > $LOG 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 60
done
echo EXIT $rc >> $LOG
