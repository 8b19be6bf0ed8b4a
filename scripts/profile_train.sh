#!/bin/bash
# rocprofv3 kernel statistics of the training bench (run on the GPU box).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run -- \
  python3 bench_train.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_train.log 2>&1
rc=$?
echo "rocprofv3 rc=$rc"
f=$(find gpurun_out/prof_train -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && head -30 "$f"
exit $rc
