# Round 6: HEAD (LDS-staged split-f16 pair, fused per-ray sums, enc_d per ray): the training tests,
# a same-box A/B of the training step against round 5, the training PMC traffic passes and a
# rocprofv3 kernel trace of the training bench.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/d
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_autograd.py -v -s -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $O/pytest_train.log 2>&1
rc=$?; echo "train tests rc=$rc"; tail -3 $O/pytest_train.log
[ $rc -ge 124 ] && exit $rc
bash scripts/ab_train_libs.sh depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_r05.so > $O/ab_train.log 2>&1
rc=$?; cat $O/ab_train.log; [ $rc -ne 0 ] && exit $rc
PASSES="1 2 3" bash scripts/profile_pmc.sh $O/pmc train > $O/pmc.log 2>&1; echo "pmc rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run -- \
  python3 bench_train.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_train.log 2>&1
echo "rocprofv3 rc=$?"
