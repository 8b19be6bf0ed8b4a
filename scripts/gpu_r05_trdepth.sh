# Prefetch depth of the coalesced-staging split-f16 weight gradient: wgrad_h16w_kernel (default) against
# wgrad_h16tr_kernel with 2, 3 and 4 stages of loads in flight (NERFMI_WGRAD_LOADER=tr3|tr4|tr5),
# same box, alternating; the training tests under tr5 first.
mkdir -p gpurun_out/r05/trd
O=gpurun_out/r05/trd
NERFMI_WGRAD_LOADER=tr5 timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $O/pytest_train_tr5.log 2>&1
rc=$?; echo "pytest tr5 rc=$rc"; tail -2 $O/pytest_train_tr5.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in w tr3 tr4 tr5; do
    if [ $v = w ]; then E=""; else E=$v; fi
    NERFMI_WGRAD_LOADER=$E timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_${v}_$i.log 2>&1 || exit $?
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05/trd/bt_*.log")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), round(d["roofline"]["kernels_ms"]["wgrad"], 4))
PY
