#!/bin/bash
# Round 5 profiles of the training step: rocprofv3 kernel statistics of bench_train.py with the
# split-f16 weight gradient (default) and with NERFMI_WGRAD=bf16x6, then the PMC passes of the
# default step (traffic, MFMA duty, stalls).  Each step under its own time limit; stops at a crash.
ROOT=$(pwd)
mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$ROOT/gpurun_out/r05/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    stats) run stats_train_h16 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r05/stats_train_h16" -o run -- \
             python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline
           NERFMI_WGRAD=bf16x6 run stats_train_bf6 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r05/stats_train_bf6" -o run -- \
             python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline ;;
    pmc) cd "$ROOT" && PASSES="${PASSES:-1 2 3 4 5 6}" timeout -k 10 900 bash scripts/profile_pmc.sh gpurun_out/r05/pmc_train train
         echo "pmc rc=$?"; cd /tmp ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
