#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
B=depth-aware-shader-effects-for-nerf_amd/build/ab
for round in 1 2; do
  for lib in ""; do
    NERFMI_LIB=$lib timeout -k 10 300 python bench_train.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/abt.log 2>&1 || { tail -5 gpurun_out/abt.log; exit 1; }
    python -c "
import json,sys; d=json.loads(open('gpurun_out/abt.log').read().strip().split('\n')[-1])
print(sys.argv[1] or 'in-tree', round(d['value']), {k: round(v, 3) for k, v in d['roofline']['kernels_ms'].items()})" "$lib"
  done
  (cd ab_r01 && NERFMI_LIB=$PWD/../$B/libnerfmi_r01.so timeout -k 10 300 python bench_train.py --steps 20 --warmup 3 --no-cpu-baseline > ../gpurun_out/abt.log 2>&1) || { tail -5 gpurun_out/abt.log; exit 1; }
  python -c "
import json,sys; d=json.loads(open('gpurun_out/abt.log').read().strip().split('\n')[-1])
print('r01', round(d['value']), {k: round(v, 3) for k, v in d['roofline']['kernels_ms'].items()})"
done
