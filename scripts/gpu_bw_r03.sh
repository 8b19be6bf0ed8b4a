#!/bin/bash
# Round 3: the bound-scaled data-gradient kernel on the GPU box: training parity (both arithmetics),
# same-box A/B against the exact-row-maximum kernel (build/ab/libnerfmi_exact.so), kernel stats.
set -o pipefail
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_train 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_autograd.py -q -p no:cacheprovider --timeout 300 --timeout-method thread
step ab_train 900 bash scripts/ab_train_libs.sh depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_base.so depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_nostore.so depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_contig.so
ROOT=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_train" -o run -- python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_train.log" 2>&1); echo "prof_train rc=$?"

