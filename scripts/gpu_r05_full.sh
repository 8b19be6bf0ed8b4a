# Round 5 checkpoint on the GPU: the whole GPU suite, the bench line, the training kernel trace and
# the training PMC passes (traffic, MFMA duty).  Each step under its own limit; stops at a crash.
mkdir -p gpurun_out/r05
bash scripts/gpu_check.sh pytest_all bench || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/r05/pytest_gpu_full.log; cp gpurun_out/bench.log gpurun_out/r05/bench_full.log
bash scripts/gpu_r05_prof.sh stats || exit $?
PASSES="1 2 3" bash scripts/gpu_r05_prof.sh pmc
