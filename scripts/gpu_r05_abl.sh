# Ablations of the whole-tile split-f16 weight gradient (timing only; wrong results by design):
# training-step phases of the in-tree library against each ablation build, 3 rounds, same box.
mkdir -p gpurun_out/r05
L=depth-aware-shader-effects-for-nerf_amd/build/ab
bash scripts/ab_train_libs.sh $L/libnerfmi_abl_NOLOAD.so $L/libnerfmi_abl_MFMA1.so $L/libnerfmi_abl_NOBIAS.so \
  $L/libnerfmi_abl_NOSPLIT.so > gpurun_out/r05/ab_wgrad_ablations.log 2>&1
rc=$?; cat gpurun_out/r05/ab_wgrad_ablations.log; exit $rc
