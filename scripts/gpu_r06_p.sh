# Round 6: (1) the upper bound of hiding the weight-gradient reductions: a timing-only build without
# any wgrad_reduce_kernel launch (wrong gradients, never shipped), same-box A/B of the training step;
# (2) the render at HEAD against round 5's library, same box (bench.py frame workload).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/p
mkdir -p $O
A=depth-aware-shader-effects-for-nerf_amd/build/ab
bash scripts/ab_train_libs.sh $A/libnerfmi_noreduce.so > $O/ab_train_noreduce.log 2>&1
rc=$?; cat $O/ab_train_noreduce.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_bench.sh $A/libnerfmi_r05.so > $O/ab_render_head_vs_r05.log 2>&1
rc=$?; cat $O/ab_render_head_vs_r05.log; exit $rc
