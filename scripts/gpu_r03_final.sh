#!/bin/bash
# Round 3 end-of-round check on the GPU box: the whole GPU suite and smoke, both benches, rocprofv3
# kernel stats of the render and the training bench, PMC passes of the training bench.
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
ROOT=$(pwd)
step pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
step bench_train 300 python bench_train.py --steps 20 --warmup 3
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_render_final" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof_render_final.log" 2>&1); echo "prof_render rc=$?"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_train_final" -o run -- python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_train_final.log" 2>&1); echo "prof_train rc=$?"
export PASSES="1 2 3"
STEPS=3 WARMUP=1 timeout -k 10 600 bash scripts/profile_pmc.sh gpurun_out/pmc_train_final train; echo "pmc_train rc=$?"
