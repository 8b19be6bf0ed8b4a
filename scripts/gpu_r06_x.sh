# Round 6: after the trainer's stream-switch removal: training, autograd and checkpoint GPU tests, smoke.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/x
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_autograd.py tests/test_gpu_checkpoint.py -v \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_train.log 2>&1
rc=$?; echo "train tests rc=$rc"; tail -2 $O/pytest_train.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -1 $O/smoke.log; exit $(( rc > rc2 ? rc : rc2 ))
