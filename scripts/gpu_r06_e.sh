# Round 6: the 16x16x32 render MLP (mlp16s_kernel).  Render parity tests first (stop on failure), then
# the same-box A/B of bench.py's render against the 32x32 kernel's library (build/ab/libnerfmi_r06tile32.so).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py -x -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread > $O/pytest_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -5 $O/pytest_parity.log
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_bench.sh depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_r06tile32.so > $O/ab_render.log 2>&1
rc=$?; cat $O/ab_render.log; exit $rc
