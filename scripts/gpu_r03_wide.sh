#!/bin/bash
# Round 3: the one-wave-per-SIMD 256x256 weight-gradient kernel (build/ab/libnerfmi_wide.so):
# training parity tests against it, then a same-box A/B of the training step against the in-tree build.
set -o pipefail
mkdir -p gpurun_out
AB=depth-aware-shader-effects-for-nerf_amd/build/ab
NERFMI_LIB=$AB/libnerfmi_wide.so timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_autograd.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_wide.log 2>&1; rc=$?; echo "pytest_wide rc=$rc"; tail -3 gpurun_out/pytest_wide.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 900 bash scripts/ab_train_libs.sh $AB/libnerfmi_wide.so $AB/libnerfmi_onestream.so > gpurun_out/ab_wide.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab_wide.log
