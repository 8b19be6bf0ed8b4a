#!/bin/bash
# Round 3: LDS-DMA operand staging for the 256-column weight gradient (build/ab/libnerfmi_dma.so,
# -DNERF_WG_DMA): training, accuracy and autograd GPU tests against that library, then a same-box
# A/B (in-tree, round-start train.hip, DMA) and a kernel trace of the DMA build.
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
DMA=depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_dma.so
ORIG=depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_orig.so
NERFMI_LIB=$DMA timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_accuracy.py tests/test_gpu_autograd.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_dma.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_dma.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 900 bash scripts/ab_train_libs.sh $ORIG $DMA > gpurun_out/ab_dma.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab_dma.log
(cd /tmp && export TMPDIR=/tmp && NERFMI_LIB="$ROOT/$DMA" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_dma" -o run -- python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_dma.log" 2>&1); echo "prof rc=$?"
