#!/bin/bash
# End-of-round check on the GPU box: every GPU test, smoke, the render bench with its CPU baseline,
# rocprofv3 kernel stats of the same bench, the training bench.  Each GPU step under its own time
# limit; the script stops at the first crash / abort / timeout (status >= 124).
set -o pipefail
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 5 --warmup 1
ROOT=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_final" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof_final.log" 2>&1); echo "prof_final rc=$?"
step bench_train 600 python bench_train.py --steps 20 --warmup 3
