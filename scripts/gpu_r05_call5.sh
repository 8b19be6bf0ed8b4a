mkdir -p gpurun_out/r05
timeout -k 10 300 python -u scripts/diag_dir_grads.py > gpurun_out/r05/diag_dir_grads.log 2>&1; echo "diag rc=$?"; tail -30 gpurun_out/r05/diag_dir_grads.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -k "chunked or param_grads or f7 or records or deterministic or production" -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05/pytest_head3.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r05/pytest_head3.log
[ $rc -ge 124 ] && exit $rc
L=depth-aware-shader-effects-for-nerf_amd/build/ab
bash scripts/ab_train_libs.sh $PWD/$L/libnerfmi_head3gemm.so $PWD/$L/libnerfmi_pesep.so $PWD/$L/libnerfmi_clen2k.so 2>&1 | tee gpurun_out/r05/ab_head3_pe_clen2k.log
