# Round 6: the 16-byte row stores with soffset 0 (the compiler pads the store-data wait states; the
# training-determinism failure of the forward loop split, scripts/diag_train_det.py).  Determinism
# (twice), the divergence diagnostic, the training tests, then a same-box A/B of the training step
# against HEAD (r06head) and the chunk-length variants built before this fix (w4k, p2k).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/j
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -v -p no:cacheprovider --timeout 200 \
    --timeout-method thread -k "deterministic" > $O/det_$rep.log 2>&1
  rc=$?; echo "determinism $rep rc=$rc $(tail -1 $O/det_$rep.log)"
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python -u scripts/diag_train_det.py > $O/diag_train_det.log 2>&1
rc=$?; echo "diag rc=$rc"; grep -v amdgpu.ids $O/diag_train_det.log | tail -8 | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $O/pytest_train.log 2>&1
rc=$?; echo "train tests rc=$rc"; tail -3 $O/pytest_train.log
[ $rc -ne 0 ] && exit $rc
A=depth-aware-shader-effects-for-nerf_amd/build/ab
bash scripts/ab_train_libs.sh $A/libnerfmi_r06head.so $A/libnerfmi_w4k.so $A/libnerfmi_p2k.so > $O/ab_train.log 2>&1
rc=$?; cat $O/ab_train.log; exit $rc
