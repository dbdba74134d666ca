#!/bin/bash
# usage: gpuq.sh TIMEOUT 'command' LOG  -- retries only when no GPU slot was free (nothing ran, nothing charged)
T=$1; CMD=$2; LOG=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then sleep 90; continue; fi
  exit $rc
done
