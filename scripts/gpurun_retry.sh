#!/bin/bash
# Local helper: run a gpurun call, re-submitting it (up to 12 tries, 60 s apart)
# only when the service reports an infrastructure transient or no free box --
# i.e. when NOTHING ran on a GPU.  Any other outcome (pass, fail, fault,
# timeout) is returned as is and never retried.
# usage: scripts/gpurun_retry.sh <log> <timeout_s> '<command>'
LOG=$1; TO=$2; CMD=$3
for try in 1 2 3 4 5 6 7 8 9 10 11 12; do
  timeout $((TO + 1200)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient\|has no free box" "$LOG" || [ $rc -eq 3 ]; then
    echo "try $try: transient / no box, retrying" >&2
    sleep 60
    continue
  fi
  exit $rc
done
exit $rc
