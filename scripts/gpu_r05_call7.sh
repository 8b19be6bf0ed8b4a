mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py -k "matches_autograd or over_steps or production_batch" -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r05/pytest_train_tight2.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/r05/pytest_train_tight2.log | tail -5
[ $rc -ge 124 ] && exit $rc
L=depth-aware-shader-effects-for-nerf_amd/build/ab
bash scripts/ab_train_libs.sh $PWD/$L/libnerfmi_clen1k.so $PWD/$L/libnerfmi_clen4k.so $PWD/$L/libnerfmi_k64c2k.so 2>&1 | tee gpurun_out/r05/ab_clen.log
