#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool reports that nothing ran (status=transient:
# no box / slot free, or the client is backing off after an infrastructure failure), waiting as long
# as the message asks.  A call that ran -- pass or fail -- is never repeated.
# Usage: scripts/gpurun_wait.sh LOG TIMEOUT 'command'
log=$1; to=$2; cmd=$3
for i in $(seq 1 ${TRIES:-30}); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && grep -q "run 0.0s\|run Nones" "$log"; then
    w=$(grep -o "retry in [0-9]*s" "$log" | grep -o "[0-9]*" | tail -1)
    w=${w:-${WAIT:-120}}
    echo "[gpurun_wait] nothing ran (try $i), waiting $((w + 15)) s" >> "$log.tries"
    sleep $((w + 15))
    continue
  fi
  exit $rc
done
exit 3
