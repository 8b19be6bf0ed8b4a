#!/bin/bash
# Round 3: same-box A/B of the training step (in-tree, round-start train.hip, LDS-DMA weight gradient)
# and a one-stream kernel trace of the DMA build.
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
DMA=depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_dma.so
ORIG=depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_orig.so
timeout -k 10 900 bash scripts/ab_train_libs.sh $ORIG $DMA > gpurun_out/ab_dma.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab_dma.log
(cd /tmp && export TMPDIR=/tmp && NERFMI_LIB="$ROOT/${DMA%.so}1s.so" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_dma" -o run -- python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_dma.log" 2>&1); echo "prof rc=$?"
