#!/bin/bash
# Round-end measurement refresh on the GPU box: GPU tests, smoke, PMC passes (f16x3), bench with
# the CPU baseline, rocprofv3 kernel stats of the same bench command, training bench.
set -o pipefail
mkdir -p gpurun_out
scripts/gpu_check.sh pytest smoke || exit $?
STEPS=3 WARMUP=1 timeout -k 10 600 bash scripts/profile_pmc.sh gpurun_out/pmc16 f16x3 || exit $?
python scripts/summarize_pmc.py gpurun_out/pmc16 gpurun_out/pmc16_summary.json || exit $?
scripts/gpu_check.sh bench || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f16 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_f16.log 2>&1 || exit $?
scripts/gpu_check.sh bench_train bench_f32
