# Round 6: same-box A/B of the training step, HEAD against round 5's library (build/ab/libnerfmi_r05.so),
# alternating, then a rocprofv3 kernel trace of the training bench at HEAD.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/b
mkdir -p $O
bash scripts/ab_train_libs.sh depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_r05.so > $O/ab_train.log 2>&1
rc=$?; cat $O/ab_train.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run -- \
  python3 bench_train.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_train.log 2>&1
rc=$?; echo "rocprofv3 rc=$rc"
f=$(find $O/prof_train -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" $O/kernel_stats_train.csv && head -25 "$f" | cut -c1-150
exit $rc
