#!/bin/bash
# Run one gpurun call; if the harness reports an infrastructure-side transient failure (no box
# was prepared, nothing ran, nothing charged) wait and submit the same call again, up to 4
# times.  Any other outcome (including a failing command) is returned as is.
#   usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in 1 2 3 4; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" && ! grep -q "status=ok\|status=fail" "$LOG"; then
    echo "[retry] transient infrastructure failure, attempt $i" >> "$LOG.retries"
    sleep 45
    continue
  fi
  exit $rc
done
exit $rc
