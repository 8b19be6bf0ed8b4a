#!/bin/bash
# Kernel durations of the standalone weight-gradient launch (scripts/wgrad_probe.py) under each
# library given (in-tree first), from rocprofv3 kernel traces.
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/wgtrace; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for lib in "" "$@"; do
  i=$((i+1))
  (cd /tmp && NERFMI_LIB=${lib:+$ROOT/$lib} ITERS=10 LDA=${LDA:-2312} LDX=${LDX:-2400} K=${K:-256} timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/l$i -o run --output-format csv -- python3 $ROOT/scripts/wgrad_probe.py > $OUT/l$i.log 2>&1) || { tail -3 $OUT/l$i.log; exit 1; }
  python3 - "$OUT/l$i" "${lib:-in-tree}" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        d[r['Kernel_Name'].split('(')[0]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
print(sys.argv[2], {k: round(sorted(v)[len(v) // 2], 1) for k, v in d.items() if 'wgrad' in k})
PY
done
