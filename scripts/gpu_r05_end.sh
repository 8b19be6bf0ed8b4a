# Round 5, last evidence at HEAD: the GPU suite, the driver's bench command (plain), smoke.
mkdir -p gpurun_out/r05/end5
O=gpurun_out/r05/end5
bash scripts/gpu_check.sh pytest_all || exit $?
cp gpurun_out/pytest_gpu.log $O/pytest_gpu.log
grep -q "FAILED" $O/pytest_gpu.log && { echo "suite not green"; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_check.sh smoke
cp gpurun_out/smoke.log $O/smoke.log
