# Round 6: the barrier-free split-f16 pair kernel.  Training tests (weight-gradient paths), then a
# same-box A/B of the training step: HEAD / HEAD without the fused per-ray sums / round 5, alternating;
# then a rocprofv3 kernel trace of the training bench at HEAD.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "pe_columns or small_rows or records or param_grads or production_batch or deterministic or over_steps" > $O/pytest_train.log 2>&1
rc=$?; echo "train tests rc=$rc"; tail -3 $O/pytest_train.log
[ $rc -ge 124 ] && exit $rc
bash scripts/ab_train_libs.sh depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_nofuse.so \
  depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_r05.so > $O/ab_train.log 2>&1
rc=$?; cat $O/ab_train.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run -- \
  python3 bench_train.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_train.log 2>&1
echo "rocprofv3 rc=$?"
timeout -k 10 200 scripts/microbench/mfma_chain > $O/mfma_chain.log 2>&1; echo "mfma_chain rc=$?"; cat $O/mfma_chain.log
