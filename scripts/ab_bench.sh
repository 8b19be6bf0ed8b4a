#!/bin/bash
# A/B of library builds on one box: alternates `python bench.py` between the in-tree library and
# each NERFMI_LIB given, twice, and prints value and per-pass MLP times.
#   bash scripts/ab_bench.sh depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_X.so ...
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for lib in "" "$@"; do
    NERFMI_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-train --no-f32 > gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
    python -c "
import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().split('\n')[-1])
print(sys.argv[1] or 'in-tree', round(d['value']), {k: round(v, 2) for k, v in d['roofline']['avg_launch_ms_by_pass'].items()})" "$lib"
  done
done
