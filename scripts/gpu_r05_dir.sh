# The dir/density weight gradient on the two-workgroups-per-CU kernel (160 of 256 rows kept; default)
# against wgrad_h16w_kernel<5> (NERFMI_WGRAD_DIR_HALF=0), and the rgb head on stream B (NERFMI_HEAD3_B=1):
# training tests first, then alternating training benches, then a kernel trace.
mkdir -p gpurun_out/r05/dir
O=gpurun_out/r05/dir
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_train.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3 4; do
  timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_dh_$i.log 2>&1 || exit $?
  NERFMI_WGRAD_DIR_HALF=0 timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_dw_$i.log 2>&1 || exit $?
  NERFMI_HEAD3_B=1 timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_dhb_$i.log 2>&1 || exit $?
done
python - <<'PY'
import json, glob, collections
m = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r05/dir/bt_*.log")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    m[f.split("/")[-1].rsplit("_", 1)[0]].append(d["value"])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), round(d["roofline"]["kernels_ms"]["wgrad"], 4))
for k, v in m.items(): print(k, round(sum(v) / len(v)))
PY
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
NERFMI_HEAD3_B=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/stats" -o run -- python3 "$R/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/$O/stats.log" 2>&1
echo "rocprof rc=$?"
