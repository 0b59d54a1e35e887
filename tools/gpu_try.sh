#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool has no free box (gpurun exit 3: nothing ran, nothing
# charged).  Any other outcome -- success, a failing command, a refusal -- ends the loop.
#   tools/gpu_try.sh <log> <timeout-seconds> '<command>'
log=$1; t=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$log"; then exit $rc; fi
  echo "[gpu_try] no box (attempt $i), retrying in 90 s" >> "$log.tries"
  sleep 90
done
exit 3
