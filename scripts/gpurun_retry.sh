#!/bin/bash
# local helper (runs here, not on the box): retry a gpurun call while the pool has no free slot or box (transient,
# nothing charged); never retries a call whose command ran
LOG=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" && ! grep -q "run [1-9]" "$LOG"; then
    echo "[retry $i] transient, waiting" >> "$LOG.retries"; sleep 180; continue
  fi
  exit $rc
done
