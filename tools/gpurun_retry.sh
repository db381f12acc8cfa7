#!/bin/bash
# Re-submit a gpurun call only when the box never ran it (status=transient:
# "stopped responding while being prepared"); any other outcome is final.
# Usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for attempt in 1 2 3 4; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  if ! grep -q "status=transient" "$LOG"; then exit 0; fi
  echo "transient (attempt $attempt), waiting" >> "$LOG.retries"
  sleep 90
done
