# Round 6: bisect the f16x3 determinism failure seen with the in-tree build (forward loop split + rgb
# head launch writing the per-ray head sums): the 25-step determinism test twice per library.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/h
mkdir -p $O
A=depth-aware-shader-effects-for-nerf_amd/build/ab
for lib in "" $A/libnerfmi_splitonly.so $A/libnerfmi_r06head.so; do
  for rep in 1 2; do
    name=$(basename "${lib:-in-tree}" .so)_$rep
    NERFMI_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -v -p no:cacheprovider --timeout 200 \
      --timeout-method thread -k "deterministic and f16x3" > $O/det_$name.log 2>&1
    rc=$?; echo "$name rc=$rc $(tail -1 $O/det_$name.log)"
    [ $rc -ge 124 ] && exit $rc
  done
done
exit 0
