#!/bin/bash
# Round 3 closing check of the in-tree build (four-wave reduction, eight loads in flight): the whole
# GPU suite and smoke, both benches; then the same-box A/B of the training step against the
# round-start train.hip and the LDS-DMA weight-gradient build, and a one-stream trace of the latter.
set -o pipefail
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
ROOT=$(pwd)
DMA=depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_dma.so
ORIG=depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_orig.so
step pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
step bench_train 300 python bench_train.py --steps 20 --warmup 3
step ab_dma 900 bash scripts/ab_train_libs.sh $ORIG $DMA
cat gpurun_out/ab_dma.log
(cd /tmp && export TMPDIR=/tmp && NERFMI_LIB="$ROOT/${DMA%.so}1s.so" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_dma" -o run -- python3 "$ROOT/bench_train.py" --steps 10 --warmup 2 --no-cpu-baseline > "$ROOT/gpurun_out/prof_dma.log" 2>&1); echo "prof rc=$?"
