#!/bin/bash
# Dev: one gpurun call; re-submits ONLY when the infrastructure refused it before anything ran
# (status=transient / no box / backing off -- nothing executed, nothing charged).  A command that ran
# and failed is never re-run.   usage: tools/dev/gpucall.sh <log> <timeout_s> '<command>'
log=$1; to=$2; cmd=$3
for attempt in 1 2 3 4 5 6 7 8; do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && ! grep -q "status=ok" "$log"; then
    if grep -qE "run [1-9][0-9.]*s of limit" "$log"; then break; fi   # something ran: do not repeat it
    sleep $((30 * attempt)); continue
  fi
  if [ $rc -eq 3 ]; then sleep $((30 * attempt)); continue; fi
  break
done
echo "gpucall rc=$rc attempts=$attempt" >> "$log"
tail -6 "$log"
