# A/B of the grouped hidden-layer weight gradient (wgrad_h16g_kernel + one grouped reduction, default)
# against seven per-layer launches (NERFMI_WGRAD_GROUP=0): the training tests first, then alternating
# training benches, then a kernel trace of each.
mkdir -p gpurun_out/r05/group
O=gpurun_out/r05/group
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py -x -v -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_train.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_g_$i.log 2>&1 || exit $?
  NERFMI_WGRAD_GROUP=0 timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_u_$i.log 2>&1 || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05/group/bt_*.log")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), round(d["roofline"]["kernels_ms"]["wgrad"], 4))
PY
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/stats_g" -o run -- python3 "$R/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/$O/stats_g.log" 2>&1
echo "rocprof rc=$?"
