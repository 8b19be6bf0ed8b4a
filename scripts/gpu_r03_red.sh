#!/bin/bash
# Round 3: eight-part weight-gradient reduction: training GPU tests, a same-box A/B against the
# four-part build, and a kernel trace of the training bench.
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_autograd.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_red.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_red.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 700 bash scripts/ab_train_libs.sh depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_red4.so > gpurun_out/ab_red.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab_red.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_red" -o run -- python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_red.log" 2>&1); echo "prof rc=$?"
