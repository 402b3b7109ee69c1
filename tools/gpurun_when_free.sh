#!/bin/bash
# Submit one gpurun call, re-submitting only while the pool answers "no slot / no box free"
# (exit 3 or status=transient: nothing ran, nothing was charged), at most TRIES times, 2 min
# apart.  A call that ran -- whatever its exit status -- is never repeated.
#   tools/gpurun_when_free.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3; TRIES=${TRIES:-10}
for i in $(seq 1 "$TRIES"); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG"; then
    exit $rc
  fi
  sleep 120
done
exit 3
