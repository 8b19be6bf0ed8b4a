# Round 6: the render kernel's side VALU from MFMA gap 5 (in-tree): render parity and shard tests; then
# the training kernels' side VALU from gap 2 / 3 (stream16.h kValuGap0; tg2 / tg3), same-box A/B of the
# training step.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/r
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py -x -v -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/pytest_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $O/pytest_parity.log; [ $rc -ne 0 ] && exit $rc
A=depth-aware-shader-effects-for-nerf_amd/build/ab
bash scripts/ab_train_libs.sh $A/libnerfmi_tg2.so $A/libnerfmi_tg3.so > $O/ab_train_vgap.log 2>&1
rc=$?; cat $O/ab_train_vgap.log; exit $rc
