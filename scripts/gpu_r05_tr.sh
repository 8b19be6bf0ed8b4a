# A/B of the split-f16 weight-gradient loaders: wgrad_h16tr_kernel (NERFMI_WGRAD_LOADER=tr, 16-byte
# coalesced loads, transposed LDS reads) against wgrad_h16w_kernel (dword loads).  Training tests
# under tr first; then alternating training benches; then kernel stats of each.
mkdir -p gpurun_out/r05/tr
O=gpurun_out/r05/tr
NERFMI_WGRAD_LOADER=tr timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $O/pytest_train_tr.log 2>&1
rc=$?; echo "pytest tr rc=$rc"; tail -2 $O/pytest_train_tr.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_w_$i.log 2>&1 || exit $?
  NERFMI_WGRAD_LOADER=tr timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_tr_$i.log 2>&1 || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05/tr/bt_*.log")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), round(d["roofline"]["kernels_ms"]["wgrad"], 4))
PY
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/stats_w" -o run -- python3 "$R/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/$O/stats_w.log" 2>&1 || exit $?
NERFMI_WGRAD_LOADER=tr timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/stats_tr" -o run -- python3 "$R/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/$O/stats_tr.log" 2>&1
echo "rocprof rc=$?"
