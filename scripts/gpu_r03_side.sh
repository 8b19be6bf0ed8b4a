#!/bin/bash
# Round 3: transposed packing on a side stream in the Trainer: training GPU tests, then a same-box A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_checkpoint.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_side.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_side.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 700 bash scripts/ab_train_env.sh NERFMI_PACKT_SIDE=0 > gpurun_out/ab_side.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab_side.log
