# Round 6: the training forward without spills (layers 4 and 7 outside the layer loop) and the rgb
# head's launch writing the per-ray head sums (block_head_sums_kernel folded in).  Training tests
# (stop on failure), then a same-box A/B of the training step: in-tree / HEAD's train.hip with the new
# forward (splitonly) / HEAD (r06head) / 4,096-sample whole-tile chunks (w4k) / 2,048-sample pair
# chunks (p2k); the last two are built on splitonly.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $O/pytest_train.log 2>&1
rc=$?; echo "train tests rc=$rc"; tail -3 $O/pytest_train.log
[ $rc -ne 0 ] && exit $rc
A=depth-aware-shader-effects-for-nerf_amd/build/ab
bash scripts/ab_train_libs.sh $A/libnerfmi_splitonly.so $A/libnerfmi_r06head.so $A/libnerfmi_w4k.so $A/libnerfmi_p2k.so \
  > $O/ab_train.log 2>&1
rc=$?; cat $O/ab_train.log; exit $rc
