#!/bin/bash
# Retries a gpurun call only while the infrastructure reports a transient failure before the
# command ran (no box / box not prepared); never re-runs a command that actually ran.
# usage: tools/gpurun_retry.sh <timeout> '<command>' <logfile>
T=$1; CMD=$2; LOG=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" && grep -q "run 0.0s\|run Nones" "$LOG"; then
    sleep 60; continue
  fi
  if [ $rc -eq 3 ]; then sleep 60; continue; fi
  break
done
tail -4 "$LOG"
