# Round 6: where two identically seeded trainers first diverge (scripts/diag_train_det.py), in-tree and HEAD.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/i
mkdir -p $O
H=depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_r06head.so
for lib in "" $H; do
  name=$(basename "${lib:-in-tree}" .so)
  NERFMI_LIB=$lib timeout -k 10 300 python -u scripts/diag_train_det.py > $O/det_$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids $O/det_$name.log | tail -12 | cut -c1-600
  [ $rc -ne 0 ] && exit $rc
done
exit 0
