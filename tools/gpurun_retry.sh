#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool reports "no box free" (exit 3: nothing ran,
# nothing charged).  Any other exit (including a failed or faulted command) ends the loop.
# usage: tools/gpurun_retry.sh LOGFILE TIMEOUT_S 'command'
log=$1; tmo=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$tmo" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "rc=$rc" >> "$log"; exit $rc; fi
  sleep 120
done
echo "gave up (no box)" >> "$log"
