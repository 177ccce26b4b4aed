#!/bin/bash
# gpurun with retries on infrastructure transients only (status=transient: nothing ran, nothing
# charged).  Any other outcome -- ok, a failing command, a refusal -- ends it.  Usage:
#   tools/gpr.sh LOG TIMEOUT 'command'
log=$1; to=$2; shift 2
for i in $(seq 1 12); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  grep -q "status=transient" "$log" || exit 0
  sleep 60
done
