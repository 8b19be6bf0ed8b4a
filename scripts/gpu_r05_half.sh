# Two workgroups per CU for the hidden layers' weight gradients (wgrad_h16h_kernel<NS>, NERFMI_WGRAD_HALF=2|3)
# against wgrad_h16w_kernel: the training tests under each first, then alternating training benches
# and a kernel trace of the better one.
mkdir -p gpurun_out/r05/half
O=gpurun_out/r05/half
for v in 3 2; do
  NERFMI_WGRAD_HALF=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest_train_h$v.log 2>&1
  rc=$?; echo "pytest h$v rc=$rc"; tail -2 $O/pytest_train_h$v.log
  [ $rc -ne 0 ] && exit $rc
done
for i in 1 2 3; do
  for v in w 2 3; do
    if [ $v = w ]; then E=""; else E=$v; fi
    NERFMI_WGRAD_HALF=$E timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_${v}_$i.log 2>&1 || exit $?
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05/half/bt_*.log")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), round(d["roofline"]["mfma"]["achieved"] if "mfma" in d["roofline"] else 0, 1), round(d["roofline"]["kernels_ms"]["wgrad"], 4))
PY
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
NERFMI_WGRAD_HALF=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/stats_h3" -o run -- python3 "$R/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/$O/stats_h3.log" 2>&1
echo "rocprof rc=$?"
