# Round 6: the checkpoint test's two renders taken apart (scripts/diag_ckpt_render.py), in-tree and HEAD~1.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/m
mkdir -p $O
for lib in "" depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_r06head.so depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_r05.so; do
  name=$(basename "${lib:-in-tree}" .so)
  NERFMI_LIB=$lib timeout -k 10 300 python -u scripts/diag_ckpt_render.py > $O/ckpt_render_$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; grep -v "amdgpu.ids\|Warning\|warn" $O/ckpt_render_$name.log | tail -24 | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
done
exit 0
