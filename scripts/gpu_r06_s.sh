# Round 6: the ray-path parameter-gradient test with N = 32 added (one ray per 32-sample block on the
# fused per-ray sums), both arithmetics.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/s
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -v -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "param_grads_ray_path" > $O/pytest_ray_path.log 2>&1
rc=$?; echo "ray path rc=$rc"; tail -3 $O/pytest_ray_path.log; exit $rc
