mkdir -p gpurun_out/r05/diag
DIAG_SAVE=gpurun_out/r05/diag timeout -k 10 300 python -u scripts/diag_dir_grads.py > gpurun_out/r05/diag_dir_grads3.log 2>&1; echo "diag rc=$?"; ls -la gpurun_out/r05/diag
