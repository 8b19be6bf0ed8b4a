#!/bin/bash
# PMC passes over the standalone wgrad launch (scripts/wgrad_probe.py), one counter group per run.
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_wgrad; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
i=0
for group in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  ITERS=5 timeout -s KILL 120 rocprofv3 --pmc $group --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 $ROOT/scripts/wgrad_probe.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float); n = collections.defaultdict(int)
for f in glob.glob('/root/repo/gpurun_out/pmc_wgrad/p*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'wgrad_bf' in r['Kernel_Name']:
            tot[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
for k in sorted(tot): print(f"{k:28s} {tot[k]/max(n[k],1):16.1f}  (per dispatch, {n[k]} rows)")
PY
