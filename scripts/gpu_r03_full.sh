#!/bin/bash
# Round 3: the whole GPU suite, a same-box A/B of the training step (in-tree = two-stream parameter
# gradients; onestream; whole = 8-wave 256x256 workgroups), both benches and a training kernel trace.
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
step pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread
step ab_train 900 bash scripts/ab_train_libs.sh $AB/libnerfmi_onestream.so $AB/libnerfmi_whole.so
step bench_train 300 python bench_train.py --steps 20 --warmup 3
step bench 300 python bench.py --steps 5 --warmup 1
ROOT=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_train4" -o run -- python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_train4.log" 2>&1); echo "prof_train rc=$?"
