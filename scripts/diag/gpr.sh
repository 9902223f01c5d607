#!/bin/bash
# gpurun with retries ONLY when nothing ran (status=transient: no box / slot / infra backoff).
# usage: gpr.sh <log> <timeout> <cmd>
LOG=$1; TO=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG"; then
    w=$(grep -o "retry in [0-9]*s" "$LOG" | grep -o "[0-9]*" | head -1); w=${w:-150}
    echo "transient (try $i), sleeping $((w + 15))s" >> "$LOG.retries"
    sleep $((w + 15)); continue
  fi
  exit $rc
done
exit 3
