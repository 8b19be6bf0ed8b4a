#!/bin/bash
# Round 3: timing-only ablations of the 256x256 weight-gradient kernel inside the training step
# (results wrong by construction): no a loads, no x loads, neither, no bf16 split.
set -o pipefail
mkdir -p gpurun_out
AB=depth-aware-shader-effects-for-nerf_amd/build/ab
timeout -k 10 900 bash scripts/ab_train_libs.sh $AB/libnerfmi_noaload.so $AB/libnerfmi_noxload.so $AB/libnerfmi_noload.so $AB/libnerfmi_nosplit.so > gpurun_out/ab_ablate.log 2>&1; echo "ablate rc=$?"; cat gpurun_out/ab_ablate.log
