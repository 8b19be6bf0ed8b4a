# Round 6, first GPU call: the training tests with their prints (branch-flip bounds, small-row
# precision, the f32 PE-column check), the whole GPU suite, and the training bench at HEAD (its CPU
# baseline now on the 4,096-ray batch).
O=gpurun_out/r06/a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "flips or matches_autograd or small_rows or pe_columns or over_steps or production_batch or records or saves_are or ray_path" > $O/pytest_train.log 2>&1
rc=$?; echo "train tests rc=$rc"; tail -3 $O/pytest_train.log
[ $rc -ge 124 ] && exit $rc
bash scripts/gpu_check.sh pytest_all || exit $?
cp gpurun_out/pytest_gpu.log $O/pytest_gpu.log
timeout -k 10 300 python bench_train.py --steps 20 > $O/bench_train.log 2>&1; rc=$?; echo "bench_train rc=$rc"
tail -1 $O/bench_train.log | cut -c1-400
