#!/bin/bash
# gpurun_retry.sh OUTFILE TIMEOUT 'command': retries only while the pool has no free box (status
# transient, nothing ran, nothing charged); any run that started is never retried.
out=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  if [ "$st" != "transient" ]; then exit 0; fi
  echo "[retry $i: pool busy]" >> "$out.retries"
  sleep 120
done
