# Chained chunk reductions (each wgrad_h16h_kernel launch runs its stream's previous reduction; default)
# against one reduction launch per GEMM (NERFMI_WGRAD_CHAIN=0): training tests, alternating training
# benches, a kernel trace.
mkdir -p gpurun_out/r05/chain
O=gpurun_out/r05/chain
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_train.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3 4; do
  timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_c_$i.log 2>&1 || exit $?
  NERFMI_WGRAD_CHAIN=0 timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_u_$i.log 2>&1 || exit $?
done
python - <<'PY'
import json, glob, collections
m = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r05/chain/bt_*.log")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    m[f.split("/")[-1].rsplit("_", 1)[0]].append(d["value"])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), round(d["roofline"]["kernels_ms"]["wgrad"], 4))
for k, v in m.items(): print(k, round(sum(v) / len(v)))
PY
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/stats" -o run -- python3 "$R/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/$O/stats.log" 2>&1
echo "rocprof rc=$?"
