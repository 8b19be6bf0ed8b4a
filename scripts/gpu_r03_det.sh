#!/bin/bash
# Round 3: training determinism (two trainers, 25 production-size steps, bit-identical) and the
# gradient-accuracy tests on the in-tree build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_accuracy.py -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "deterministic or gradients_vs_float64 or production" > gpurun_out/pytest_det.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_det.log | tail -12
