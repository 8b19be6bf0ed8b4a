# Round 5 end-of-round evidence: the GPU suite, the bench command under rocprofv3 (kernel stats of the
# exact line the driver runs), the render PMC passes (traffic, MFMA duty) and smoke.
mkdir -p gpurun_out/r05
ROOT=$(pwd)
bash scripts/gpu_check.sh pytest_all || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/r05/pytest_gpu_final.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r05/stats_bench" -o run -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 1 > "$ROOT/gpurun_out/r05/bench_rocprof.log" 2>&1
rc=$?; echo "rocprof bench rc=$rc"; tail -1 "$ROOT/gpurun_out/r05/bench_rocprof.log" | cut -c1-400
[ $rc -ge 124 ] && exit $rc
cd "$ROOT" && PASSES="1 2 3" timeout -k 10 600 bash scripts/profile_pmc.sh gpurun_out/r05/pmc_render f16x3; echo "pmc rc=$?"
bash scripts/gpu_check.sh smoke
cp gpurun_out/smoke.log gpurun_out/r05/smoke_final.log
