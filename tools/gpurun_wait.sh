#!/bin/bash
# Run ONE gpurun call, waiting for a free GPU slot: re-submits only while
# gpurun reports status=transient (no slot / no box: nothing ran, nothing
# charged).  Any other outcome -- success, a failing command, a timeout --
# ends it.  Usage: tools/gpurun_wait.sh LOG TIMEOUT_S 'command'
LOG=$1
TO=$2
shift 2
for i in $(seq 1 30); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  grep -q "status=transient" "$LOG" || exit 0
  sleep 60
done
