#!/bin/bash
# PMC passes for the bench workload (one counter group per rocprofv3 run, as MI355X_MICROARCH.md
# prescribes: FETCH_SIZE and WRITE_SIZE do not fit one pass).  Usage (on the GPU box, repo root):
#   bash scripts/profile_pmc.sh gpurun_out/pmc [f16x3|f32|train]
set -e
OUT=${1:-gpurun_out/pmc}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
ARITH=${2:-f16x3}
if [ "$ARITH" = train ]; then   # the training step (bench_train.py, f16x3) instead of the frame render
  CMD="python3 $ROOT/bench_train.py --steps ${STEPS:-3} --warmup ${WARMUP:-1} --no-cpu-baseline"
else
  CMD="python3 $ROOT/bench.py --steps ${STEPS:-1} --warmup ${WARMUP:-0} --no-cpu-baseline --no-train --no-f32 --arith $ARITH"
fi
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  case " ${PASSES:-1 2 3 4 5 6} " in *" $i "*) ;; *) continue ;; esac
  timeout -k 10 300 rocprofv3 --pmc $group --kernel-trace -d "$ROOT/$OUT/p$i" -o run --output-format csv -- $CMD > "$ROOT/$OUT/p$i.log" 2>&1
done
