# Round 6: determinism stress at HEAD (the store-data race was timing-dependent): the 25-step
# determinism test three times (both arithmetics) and the two-trainer divergence diagnostic.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/w
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -v -p no:cacheprovider --timeout 200 \
    --timeout-method thread -k "deterministic" > $O/det_$rep.log 2>&1
  rc=$?; echo "determinism $rep rc=$rc $(tail -1 $O/det_$rep.log)"
  [ $rc -ne 0 ] && exit $rc
done
STEPS=10 timeout -k 10 300 python -u scripts/diag_train_det.py > $O/diag_train_det.log 2>&1
rc=$?; echo "diag rc=$rc"; grep -E "^step|library" $O/diag_train_det.log | cut -c1-120; exit $rc
