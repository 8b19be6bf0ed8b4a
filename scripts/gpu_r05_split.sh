# The split-only transposed pack in the training loop (default under f16x3) against the full pack
# (NERFMI_PACKT_FULL=1): training tests first, then alternating training benches.
mkdir -p gpurun_out/r05/split
O=gpurun_out/r05/split
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q -p no:cacheprovider --timeout 200 \
  --timeout-method thread > $O/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_train.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3 4; do
  timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_split_$i.log 2>&1 || exit $?
  NERFMI_PACKT_FULL=1 timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_full_$i.log 2>&1 || exit $?
done
python - <<'PY'
import json, glob, collections
m = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r05/split/bt_*.log")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    m[f.split("/")[-1].rsplit("_", 1)[0]].append(d["value"])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), {k: round(v, 3) for k, v in d["stage_ms"].items()})
for k, v in m.items(): print(k, round(sum(v) / len(v)))
PY
