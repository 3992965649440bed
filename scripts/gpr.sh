#!/bin/bash
# usage: gpr.sh LOG TIMEOUT CMD  -- retries only when gpurun reports no slot/box (rc 3), at most 12 times
LOG=$1; TO=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "rc=$rc" >> $LOG; exit $rc; fi
  sleep 90
done
echo "gave up (no slot)" >> $LOG
