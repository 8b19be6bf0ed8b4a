#!/bin/bash
# Round-4 GPU steps, each under its own time limit; stops at the first crash/abort/timeout (status
# >= 124), continues past ordinary test failures.  Usage: bash scripts/gpu_r04.sh step...
#   pytest        the whole GPU suite (one process)
#   pytest_k EXPR the GPU tests matching EXPR
#   smoke | bench | bench_train
#   ab_train LIB...   same-box A/B of the training step against NERFMI_LIB builds (scripts/ab_train_libs.sh)
#   ab_render LIB...  same-box A/B of the render bench (scripts/ab_bench.sh)
#   prof_render | prof_train   rocprofv3 --kernel-trace --stats of the benches (gpurun_out/prof_*)
#   pmc_render | pmc_train     PMC passes 1-3 (FETCH_SIZE, WRITE_SIZE, MFMA busy + clock) of the benches
#                              (scripts/profile_pmc.sh; summarise with scripts/summarize_pmc.py)
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
while [ $# -gt 0 ]; do
  step=$1; shift
  case $step in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    pytest_k) run pytest_k 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "$1"; shift ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 300 python bench.py ;;
    bench_train) run bench_train 300 python bench_train.py --steps 20 --warmup 3 ;;
    ab_train) libs=(); while [ $# -gt 0 ] && [[ $1 == *.so ]]; do libs+=("$1"); shift; done
              run ab_train 900 bash scripts/ab_train_libs.sh "${libs[@]}" ;;
    ab_render) libs=(); while [ $# -gt 0 ] && [[ $1 == *.so ]]; do libs+=("$1"); shift; done
               run ab_render 900 bash scripts/ab_bench.sh "${libs[@]}" ;;
    prof_render) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_render" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/prof_render.log" 2>&1); rc=$?; echo "prof_render rc=$rc"; [ $rc -ge 124 ] && exit $rc ;;
    prof_train) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_train" -o run -- python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_train.log" 2>&1); rc=$?; echo "prof_train rc=$rc"; [ $rc -ge 124 ] && exit $rc ;;
    pmc_render) PASSES="1 2 3" STEPS=1 WARMUP=0 run pmc_render 600 bash scripts/profile_pmc.sh gpurun_out/pmc_render f16x3 ;;
    pmc_train) PASSES="1 2 3" STEPS=3 WARMUP=1 run pmc_train 600 bash scripts/profile_pmc.sh gpurun_out/pmc_train train ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
