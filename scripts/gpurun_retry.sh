#!/bin/bash
# gpurun_retry.sh OUTFILE TIMEOUT 'command': retries only while the pool has no free box (status
# transient, nothing ran, nothing charged); any run that started is never retried.  The status is read
# from gpurun's own output (gpurun_out/.last_call.json is not rewritten by a call that never ran).
out=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  if ! grep -q "status=transient" "$out"; then exit 0; fi
  echo "[retry $i: pool busy]" >> "$out.retries"
  sleep 120
done
