#!/bin/bash
# gpurun wrapper: re-submits ONLY when the infrastructure reports a transient
# failure before anything ran (status=transient / exit 3). Never re-runs a
# command that actually ran on the GPU.  Usage: gpurun_retry.sh <log> <timeout> <cmd>
log=$1; to=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then
    echo "[retry] transient infrastructure failure ($i), waiting" >> "$log.retries"
    sleep 150
    continue
  fi
  exit $rc
done
exit $rc
