# The transposed weight pack in three launches (statsT16_kernel: the three statistics passes with a
# last-block finalize; the constant slots zeroed by packT_kernel): training tests, then alternating
# training benches against the previous library (build/ab/libnerfmi_prevT.so), then a kernel trace.
mkdir -p gpurun_out/r05/packt
O=gpurun_out/r05/packt
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q -p no:cacheprovider --timeout 200 \
  --timeout-method thread > $O/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_train.log
[ $rc -ne 0 ] && exit $rc
L=depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_prevT.so
for i in 1 2 3 4; do
  timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_new_$i.log 2>&1 || exit $?
  NERFMI_LIB=$L timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_old_$i.log 2>&1 || exit $?
done
python - <<'PY'
import json, glob, collections
m = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r05/packt/bt_*.log")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    m[f.split("/")[-1].rsplit("_", 1)[0]].append(d["value"])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), {k: round(v, 3) for k, v in d["stage_ms"].items()})
for k, v in m.items(): print(k, round(sum(v) / len(v)))
PY
