#!/bin/bash
# Round 5: the split-f16 weight gradient on the GPU -- training parity + accuracy tests, then a
# same-box A/B of the training step (default h16 vs NERFMI_WGRAD=bf16x6), alternating.
mkdir -p gpurun_out/r05
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r05/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -4 "gpurun_out/r05/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    tests) run pytest_train 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_accuracy.py tests/test_gpu_autograd.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    ab) for i in 1 2 3; do
          run bt_h16_$i 300 python bench_train.py --steps 30 --warmup 5 --no-cpu-baseline
          NERFMI_WGRAD=bf16x6 run bt_bf6_$i 300 python bench_train.py --steps 30 --warmup 5 --no-cpu-baseline
        done
        grep -ho '"value": [0-9.]*\|"wgrad": [0-9.]*' gpurun_out/r05/bt_*.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
