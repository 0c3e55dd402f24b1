#!/bin/bash
# Re-submit a gpurun call ONLY when the box could not be prepared (status=transient: nothing ran,
# nothing charged).  Any other outcome -- including a failing command -- is returned as is.
LOG=$1; shift
for attempt in 1 2 3 4; do
  /usr/local/graft/bin/gpurun "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient\|rc=3\|no box or slot" "$LOG" && ! grep -q "status=ok" "$LOG"; then
    sleep $((30 * attempt)); continue
  fi
  exit $rc
done
exit $rc
