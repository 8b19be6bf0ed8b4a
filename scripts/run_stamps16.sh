# Runs the mlp16 stamp diagnostics built beforehand (scripts/microbench/mlp16_stamps_<variant>).
set -o pipefail
for v in ${STAMP_VARIANTS:-base}; do
  echo "=== $v"
  timeout -k 10 60 ./scripts/microbench/mlp16_stamps_$v > gpurun_out/stamps16_$v.log 2>&1 || { echo "rc=$?"; cat gpurun_out/stamps16_$v.log; exit 1; }
  cat gpurun_out/stamps16_$v.log
done
