# Round 6: the rgb head's weight-gradient launch (with the per-ray head sums) right after the pair on
# stream B instead of after the dir/density launch: training tests, then a same-box A/B of the training
# step against the previous build (build/ab/libnerfmi_r06final.so).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "param_grads or deterministic or production_batch or over_steps or records" > $O/pytest_train.log 2>&1
rc=$?; echo "train tests rc=$rc"; tail -2 $O/pytest_train.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_train_libs.sh depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_r06final.so > $O/ab_train_head_early.log 2>&1
rc=$?; cat $O/ab_train_head_early.log; exit $rc
