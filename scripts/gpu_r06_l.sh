# Round 6 evidence at HEAD: the bench line (driver command), rocprofv3 kernel traces of bench.py and
# bench_train.py, and the PMC traffic passes (render f16x3, training).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/lf
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 $O/bench.log; echo
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run -- \
  python3 bench.py --steps 5 --warmup 1 > $O/prof_bench.log 2>&1
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run -- \
  python3 bench_train.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_train.log 2>&1
rc=$?; echo "rocprof train rc=$rc"; [ $rc -ne 0 ] && exit $rc
PASSES="1 2 3" bash scripts/profile_pmc.sh $O/pmc_f16x3 f16x3 > $O/pmc_f16x3.log 2>&1; rc=$?; echo "pmc render rc=$rc"
[ $rc -ne 0 ] && exit $rc
PASSES="1 2 3" bash scripts/profile_pmc.sh $O/pmc_train train > $O/pmc_train.log 2>&1; rc=$?; echo "pmc train rc=$rc"
exit $rc
