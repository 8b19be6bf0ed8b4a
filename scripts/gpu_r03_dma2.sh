#!/bin/bash
# Round 3: which build fails test_gradients_vs_float64[f32-trained]: in-tree (four-part reduction),
# round-start train.hip, and the LDS-DMA weight-gradient build.
set -o pipefail
mkdir -p gpurun_out
for lib in "" depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_orig.so depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_dma.so; do
  n=$(basename "${lib:-in-tree}")
  NERFMI_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_accuracy.py -k gradients_vs_float64 -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_g64_$n.log 2>&1; rc=$?
  echo "$n rc=$rc"; grep -E "passed|failed|AssertionError: \(" gpurun_out/pytest_g64_$n.log | head -6
  [ $rc -ge 124 ] && exit $rc
done
exit 0
