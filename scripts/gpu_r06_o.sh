# Round 6: render-MLP time per sample against launch size with packed random-init weights, the 16x16x32
# kernel (in-tree) against round 5's 32x32 (libnerfmi_r05.so), alternating twice on one box
# (scripts/render_size_sweep.py); then the repeatability diagnostics with packed weights.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/o2
mkdir -p $O
for rep in 1 2; do
  for lib in "" depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_r05.so; do
    NERFMI_LIB=$lib timeout -k 10 200 python -u scripts/render_size_sweep.py >> $O/sweep.log 2>&1
    rc=$?; echo "rep $rep ${lib:-in-tree} rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/sweep.log; exit $rc; }
  done
done
grep '^{' $O/sweep.log
timeout -k 10 300 python -u scripts/diag_render_det.py > $O/render_det.log 2>&1
rc=$?; echo "render det rc=$rc"; grep "differ" $O/render_det.log | tail -12; [ $rc -ne 0 ] && exit $rc
MODE=scribble REPS=10 timeout -k 10 300 python -u scripts/diag_fwd_race.py > $O/fwd_race.log 2>&1
rc=$?; echo "fwd race rc=$rc"; grep -v amdgpu.ids $O/fwd_race.log | tail -4; exit $rc
