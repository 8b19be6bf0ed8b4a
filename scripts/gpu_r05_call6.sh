mkdir -p gpurun_out/r05
timeout -k 10 300 python -u scripts/diag_dir_grads.py > gpurun_out/r05/diag_dir_grads2.log 2>&1; echo "diag rc=$?"; tail -30 gpurun_out/r05/diag_dir_grads2.log
