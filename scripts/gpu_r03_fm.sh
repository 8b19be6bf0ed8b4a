#!/bin/bash
# Round 3: timing-only emulation of feature-major block loads in the weight-gradient kernel
# (results wrong by construction) against the in-tree build and the no-load ablation; plus the new
# ray-path parameter-gradient test on the in-tree build.
set -o pipefail
mkdir -p gpurun_out
AB=depth-aware-shader-effects-for-nerf_amd/build/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -k "ray_path or generic_shapes" -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_raypath.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_raypath.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 800 bash scripts/ab_train_libs.sh $AB/libnerfmi_fmemul.so $AB/libnerfmi_noload.so > gpurun_out/ab_fm.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab_fm.log
