#!/bin/bash
# Round 3: timing-only ablations of the one-wave-per-SIMD weight-gradient kernel inside the training
# step (results wrong by construction), two-stream and one-stream.
set -o pipefail
mkdir -p gpurun_out
AB=depth-aware-shader-effects-for-nerf_amd/build/ab
timeout -k 10 1000 bash scripts/ab_train_libs.sh $AB/libnerfmi_noaload.so $AB/libnerfmi_noxload.so $AB/libnerfmi_noload.so $AB/libnerfmi_nosplit.so $AB/libnerfmi_onestream.so $AB/libnerfmi_onestream_noload.so > gpurun_out/ab_ablate2.log 2>&1; echo "ablate rc=$?"; cat gpurun_out/ab_ablate2.log
