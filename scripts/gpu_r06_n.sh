# Round 6: verdict item 4's measurement: the training forward's extra cost over the render kernel by
# timing-only ablation builds (no save stores / no mask bits / no block records / none of the three;
# never shipped), same-box A/B of the training step; then the fixed checkpoint test.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/n
mkdir -p $O
A=depth-aware-shader-effects-for-nerf_amd/build/ab
bash scripts/ab_train_libs.sh $A/libnerfmi_abl_nostore.so $A/libnerfmi_abl_nomask.so $A/libnerfmi_abl_norec.so \
  $A/libnerfmi_abl_bare.so > $O/ab_fwd_ablation.log 2>&1
rc=$?; cat $O/ab_fwd_ablation.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_checkpoint.py -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $O/ckpt.log 2>&1
rc=$?; echo "ckpt rc=$rc"; tail -3 $O/ckpt.log; exit $rc
