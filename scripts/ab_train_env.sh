#!/bin/bash
# Same-box A/B of the training step under two environments: "" (defaults) against each VAR=VALUE given, 3 rounds.
set -o pipefail
mkdir -p gpurun_out
for round in 1 2 3; do
  for e in "" "$@"; do
    env $e timeout -k 10 300 python bench_train.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/abe.log 2>&1 || { tail -5 gpurun_out/abe.log; exit 1; }
    python -c "
import json,sys; d=json.loads(open('gpurun_out/abe.log').read().strip().split('\n')[-1])
print(sys.argv[1] or 'default', round(d['value']), round(d['ms_per_step'], 3))" "$e"
  done
done
