# Small-kernel trims of the training step (pack chain in two launches, ray features on 16-ray blocks
# for small batches, the loss on the second stream, the appearance row written in place): the GPU
# suite first, then alternating training benches against the previous library (build/ab/libnerfmi_head.so,
# same Python), then a kernel trace.
mkdir -p gpurun_out/r05/fuse2
O=gpurun_out/r05/fuse2
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
L=depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_head.so
for i in 1 2 3; do
  timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_new_$i.log 2>&1 || exit $?
  NERFMI_LIB=$L timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bt_old_$i.log 2>&1 || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05/fuse2/bt_*.log")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), {k: round(v, 3) for k, v in d["stage_ms"].items()})
PY
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/stats" -o run -- python3 "$R/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/$O/stats.log" 2>&1
echo "rocprof rc=$?"
