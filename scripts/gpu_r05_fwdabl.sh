# Cost of the training forward's stores (timing-only ablation builds: no activation saves / no mask
# bits; wrong gradients) and of the transposed packing on the side stream (NERFMI_PACKT_SIDE=0):
# training-step phases, 3 rounds, same box.
mkdir -p gpurun_out/r05
L=depth-aware-shader-effects-for-nerf_amd/build/ab
bash scripts/ab_train_libs.sh $L/libnerfmi_nosaves.so $L/libnerfmi_nomasks.so > gpurun_out/r05/ab_fwd_stores.log 2>&1 || exit $?
for i in 1 2 3; do
  for v in 1 0; do
    NERFMI_PACKT_SIDE=$v timeout -k 10 120 python bench_train.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r05/bt_side$v.log 2>&1 || exit $?
    python -c "
import json,sys; d=json.loads(open('gpurun_out/r05/bt_side$v.log').read().strip().split('\n')[-1])
print('packT side=$v', round(d['value']), {k: round(v, 3) for k, v in d['stage_ms'].items()})" >> gpurun_out/r05/ab_fwd_stores.log
  done
done
cat gpurun_out/r05/ab_fwd_stores.log
