#!/bin/bash
# GPU-box validation: each step under its own time limit; stops at the first crash/abort/timeout
# (status >= 124), continues past ordinary test failures.  Usage: scripts/gpu_check.sh step...
#   steps: pytest | pytest_all | parity | pytest_train | bench | bench_f32 | bench_train | smoke
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    pytest) run pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider ;;
    pytest_all) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    pytest_new) run pytest_new 900 python -u -m pytest tests/test_gpu_autograd.py tests/test_gpu_shards.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    pytest_train) run pytest_train 600 python -m pytest tests/test_gpu_train.py -q -p no:cacheprovider ;;
    bench) run bench 600 python bench.py --steps 5 --warmup 1 ;;
    bench_f32) run bench_f32 600 python bench.py --steps 3 --warmup 1 --arith f32 --no-cpu-baseline ;;
    parity) run pytest_parity 600 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    bench_train) run bench_train 600 python bench_train.py --steps 20 --warmup 3 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
