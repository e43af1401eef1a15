#!/bin/bash
# gpurun_wait.sh CMD... — run a gpurun call, re-submitting it only while the pool
# reports no free box / slot (status "transient": nothing ran, nothing charged).
# Any other outcome (ok, failure, fault, refusal) ends the loop.
tries=${GPURUN_TRIES:-30}
for ((i = 0; i < tries; i++)); do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  st=$(python3 -c 'import json;print(json.load(open("gpurun_out/.last_call.json")).get("status",""))' 2>/dev/null)
  if [ "$st" != "transient" ]; then exit $rc; fi
  sleep 90
done
exit 3
