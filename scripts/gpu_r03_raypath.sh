#!/bin/bash
# Round 3: the ray-path parameter-gradient test and the training GPU tests on the in-tree build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_autograd.py tests/test_capi_host.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_raypath.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/pytest_raypath.log | tail -8
