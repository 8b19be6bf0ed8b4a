#!/bin/bash
# Round 3: dir_linear + density head as a 160-row GEMM on the whole-tile kernel: training GPU tests,
# then a same-box A/B of the training step against the 256-row build (build/ab/libnerfmi_dir256.so).
set -o pipefail
mkdir -p gpurun_out
AB=depth-aware-shader-effects-for-nerf_amd/build/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_autograd.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_dir160.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_dir160.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 700 bash scripts/ab_train_libs.sh $AB/libnerfmi_dir256.so > gpurun_out/ab_dir160.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab_dir160.log
