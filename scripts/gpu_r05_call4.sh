mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py -k "matches_autograd or over_steps or production_batch or records or chunked or unaligned or extreme" -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r05/pytest_train_tight.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r05/pytest_train_tight.log
if [ $rc -lt 124 ]; then bash scripts/gpu_r05_prof.sh stats; fi
