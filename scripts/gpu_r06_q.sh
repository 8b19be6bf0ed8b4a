# Round 6: the render kernel's side-work VALU starting at MFMA gap 5, 7 or 9 of a segment instead of 1
# (its bias reads, issued at the segment's start, have ~2 x 16x16x32 MFMAs of cover at gap 1): same-box
# A/B of bench.py's frame render against the in-tree build.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/q2
mkdir -p $O
A=depth-aware-shader-effects-for-nerf_amd/build/ab
bash scripts/ab_bench.sh $A/libnerfmi_vg5.so $A/libnerfmi_vg7.so $A/libnerfmi_vg9.so > $O/ab_render_vgap.log 2>&1
rc=$?; cat $O/ab_render_vgap.log; exit $rc
