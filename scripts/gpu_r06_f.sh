# Round 6: tuning variants of mlp16s_kernel, same-box A/B against the in-tree build (bench.py render).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/f
mkdir -p $O
A=depth-aware-shader-effects-for-nerf_amd/build/ab
bash scripts/ab_bench.sh $A/libnerfmi_v48.so $A/libnerfmi_v32.so $A/libnerfmi_ds0.so $A/libnerfmi_bshare.so > $O/ab_render.log 2>&1
rc=$?; cat $O/ab_render.log; exit $rc
