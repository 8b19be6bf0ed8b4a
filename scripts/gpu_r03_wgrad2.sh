#!/bin/bash
# Round 3: weight-gradient variants on the GPU box: training/autograd/accuracy GPU tests (in-tree: two
# 4-wave workgroups per chunk of the 256x256 GEMMs, per-ray sums, bound-scaled data gradient), the
# gradient-accuracy test against the exact-row-maximum build, a same-box A/B of the training step
# (whole = one 8-wave workgroup per chunk; exact; noray), and a kernel trace.
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
AB=depth-aware-shader-effects-for-nerf_amd/build/ab
step pytest_train 900 python -u -m pytest tests/test_gpu_autograd.py tests/test_gpu_train.py tests/test_gpu_accuracy.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread
NERFMI_LIB=$AB/libnerfmi_exact.so step pytest_exact 600 python -u -m pytest tests/test_gpu_accuracy.py -k gradients -v -s -p no:cacheprovider --timeout 300 --timeout-method thread
step ab_train 900 bash scripts/ab_train_libs.sh $AB/libnerfmi_whole.so $AB/libnerfmi_exact.so $AB/libnerfmi_noray.so
ROOT=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_train3" -o run -- python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_train3.log" 2>&1); echo "prof_train rc=$?"
