#!/bin/bash
# Same-box A/B of the training step: the in-tree library against each NERFMI_LIB given, 3 rounds.
set -o pipefail
mkdir -p gpurun_out
for round in 1 2 3; do
  for lib in "" "$@"; do
    NERFMI_LIB=$lib timeout -k 10 300 python bench_train.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/abt.log 2>&1 || { tail -5 gpurun_out/abt.log; exit 1; }
    python -c "
import json,sys; d=json.loads(open('gpurun_out/abt.log').read().strip().split('\n')[-1])
print(sys.argv[1].split('/')[-1] or 'in-tree', round(d['value']), {k: round(v, 3) for k, v in d['roofline']['kernels_ms'].items()})" "$lib"
  done
done
