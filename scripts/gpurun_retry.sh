#!/bin/bash
# queue a gpurun call: retry ONLY while the pool has no free slot/box (exit 3, nothing charged);
# any other outcome (success, failure, timeout) ends the loop. usage: gpurun_retry.sh OUT TIMEOUT cmd...
out=$1; t=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "$out" 2>&1; rc=$?
  if [ $rc -ne 3 ] && ! grep -q '"status": "transient"' gpurun_out/.last_call.json 2>/dev/null; then exit $rc; fi
  sleep 150
done
exit 3
