#!/bin/bash
# Round 3: per-kernel durations of the training step on one stream (build/ab/libnerfmi_onestream.so):
# the two-stream trace overlaps the parameter-gradient kernels, so their lengths alone come from here.
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
(cd /tmp && export TMPDIR=/tmp && NERFMI_LIB=$ROOT/depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_onestream.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_train_1s" -o run -- python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_train_1s.log" 2>&1); echo "prof rc=$?"
