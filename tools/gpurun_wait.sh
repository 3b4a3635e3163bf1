#!/bin/bash
# Run one gpurun call, waiting while the pool has no free box (exit 3: nothing ran, nothing charged).
# Usage: tools/gpurun_wait.sh LOG TIMEOUT_S CMD
log=$1; t=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  grep -q "no free box\|busy" "$log" || exit $rc
  sleep 150
done
exit 3
