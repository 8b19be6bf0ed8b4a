# Round 6: the render kernel's side reads one segment ahead (VALU from gap 1 in segments 1-3, gap 5 in
# segment 0): render parity and shard tests, then a same-box A/B against the gap-5 build
# (build/ab/libnerfmi_r06g5.so).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/t
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py -x -v -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/pytest_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $O/pytest_parity.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_bench.sh depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_r06g5.so > $O/ab_render_pre.log 2>&1
rc=$?; cat $O/ab_render_pre.log; exit $rc
