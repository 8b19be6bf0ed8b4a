# Round 6 evidence at HEAD: the whole GPU suite (both arithmetics) and smoke.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/kf
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -3 $O/smoke.log
exit $(( rc > rc2 ? rc : rc2 ))
