# Round 5 end-of-round evidence at the final code: the GPU suite, the bench command under rocprofv3,
# the training PMC passes (traffic of the weight-gradient phase with wgrad_h16h_kernel), a 5-pair
# A/B of the two weight-gradient kernels, and smoke.
mkdir -p gpurun_out/r05/final
ROOT=$(pwd)
O=gpurun_out/r05/final
bash scripts/gpu_check.sh pytest_all || exit $?
cp gpurun_out/pytest_gpu.log $O/pytest_gpu.log
grep -q " passed" $O/pytest_gpu.log && ! grep -q "FAILED" $O/pytest_gpu.log || { echo "suite not green"; exit 1; }
for i in 1 2 3 4 5; do
  timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_h_$i.log 2>&1 || exit $?
  NERFMI_WGRAD_HALF=0 timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_w_$i.log 2>&1 || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05/final/bt_*.log")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), round(d["roofline"]["kernels_ms"]["wgrad"], 4))
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/stats_bench" -o run -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 1 > "$ROOT/$O/bench_rocprof.log" 2>&1
rc=$?; echo "rocprof bench rc=$rc"
[ $rc -ge 124 ] && exit $rc
cd "$ROOT" && PASSES="1 2 3" timeout -k 10 600 bash scripts/profile_pmc.sh $O/pmc_train train; echo "pmc rc=$?"
bash scripts/gpu_check.sh smoke
cp gpurun_out/smoke.log $O/smoke.log
