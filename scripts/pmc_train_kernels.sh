#!/bin/bash
# Instruction-mix PMC passes over the training bench (one counter group per rocprofv3 run), summarised
# per kernel: bash scripts/pmc_train_kernels.sh [kernel-substring]
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_tk; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
i=0
for group in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $group --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 $ROOT/bench_train.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 - "${1:-backward}" <<'PY'
import csv, glob, collections, sys
tot = collections.defaultdict(float); n = collections.defaultdict(int)
for f in glob.glob('/root/repo/gpurun_out/pmc_tk/p*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if sys.argv[1] in r['Kernel_Name']:
            tot[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
for k in sorted(tot): print(f"{k:28s} {tot[k]/max(n[k],1):16.1f}  (per dispatch, {n[k]} rows)")
PY
