#!/bin/bash
# gpurun with a bounded wait for a GPU slot: retried ONLY when gpurun reports
# exit code 3 (no box or slot free right now, nothing ran, nothing charged);
# any other outcome -- success, a failing or killed GPU step -- is final.
# usage: tools/gpurun_retry.sh <log> <timeout s> '<command>'
LOG=$1; T=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  [ $rc -eq 3 ] || exit $rc
  echo "[retry] no GPU slot (rc 3), attempt $i" >> "$LOG.retries"
  sleep 150
done
exit 3
