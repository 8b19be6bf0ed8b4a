#!/bin/bash
# A/B of library builds on one box for the training step: alternates bench_train.py between the
# in-tree library and each NERFMI_LIB given, twice; prints rays/s and per-kernel ms.
#   bash scripts/ab_train.sh depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_X.so ...
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for lib in "" "$@"; do
    NERFMI_LIB=$lib timeout -k 10 300 python bench_train.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/abt.log 2>&1 || { cat gpurun_out/abt.log; exit 1; }
    python -c "
import json,sys; d=json.loads(open('gpurun_out/abt.log').read().strip().split('\n')[-1])
print(sys.argv[1] or 'in-tree', round(d['value']), {k: round(v, 3) for k, v in d['roofline']['kernels_ms'].items()})" "$lib"
  done
done
