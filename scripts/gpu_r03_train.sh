#!/bin/bash
# Round 3: training-path check on the GPU box: the autograd / training / accuracy GPU tests, a same-box
# A/B of the training step (in-tree = bound-scaled data gradient, exact-row-maximum build), PMC passes
# of the training bench (traffic, clocks), and a kernel trace.  Each step under its own limit.
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
step pytest_train 900 python -u -m pytest tests/test_gpu_autograd.py tests/test_gpu_train.py tests/test_gpu_accuracy.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread
step ab_train 600 bash scripts/ab_train_libs.sh depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_exact.so
PASSES="1 2 3" STEPS=3 WARMUP=1 step pmc_train 600 bash scripts/profile_pmc.sh gpurun_out/pmc_train train
ROOT=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_train" -o run -- python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_train.log" 2>&1); echo "prof_train rc=$?"
