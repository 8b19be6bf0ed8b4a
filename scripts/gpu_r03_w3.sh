#!/bin/bash
# Round 3: the stream waits count one more half-step of side-work stores (stream16.h): training and
# parity GPU tests, then a same-box A/B of the training step against NERF16_WAIT_STORES_2.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_autograd.py tests/test_gpu_accuracy.py tests/test_gpu_parity.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_w3.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_w3.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 700 bash scripts/ab_train_libs.sh depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_w2.so > gpurun_out/ab_w3.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab_w3.log
