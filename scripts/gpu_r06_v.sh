# Round 6: the render kernel's side VALU from gap 4 / 6 against the in-tree gap 5, same box.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/v
mkdir -p $O
A=depth-aware-shader-effects-for-nerf_amd/build/ab
bash scripts/ab_bench.sh $A/libnerfmi_g4.so $A/libnerfmi_g6.so > $O/ab_render_g46.log 2>&1
rc=$?; cat $O/ab_render_g46.log; exit $rc
