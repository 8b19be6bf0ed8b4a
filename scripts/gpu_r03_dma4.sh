#!/bin/bash
# Round 3: kink-safe test_gradients_vs_float64; the training + accuracy + autograd GPU tests in one
# process for the in-tree and the LDS-DMA builds, then a same-box A/B and a kernel trace of the DMA build.
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
DMA=depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_dma.so
ORIG=depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_orig.so
for lib in "" $DMA; do
  n=$(basename "${lib:-in-tree}")
  NERFMI_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_accuracy.py tests/test_gpu_autograd.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_seq_$n.log 2>&1; rc=$?
  echo "$n rc=$rc"; grep -E "passed|failed|AssertionError: \(" gpurun_out/pytest_seq_$n.log | head -8
  [ $rc -ne 0 ] && exit 1
done
timeout -k 10 900 bash scripts/ab_train_libs.sh $ORIG $DMA > gpurun_out/ab_dma.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab_dma.log
(cd /tmp && export TMPDIR=/tmp && NERFMI_LIB="$ROOT/${DMA%.so}1s.so" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_dma" -o run -- python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_dma.log" 2>&1); echo "prof rc=$?"
