#!/bin/bash
# Is the x2 FETCH_SIZE correction (MI355X_MICROARCH.md §HBM: exact for 16-byte-per-lane streaming
# reads) right for the weight-gradient kernels' loads (dword buffer loads of strided rows)?  Each shape
# of the training step's wgrad GEMMs runs standalone (scripts/wgrad_probe.py, the training workspace's
# row strides, 262,144 samples, operands far larger than the 256 MiB Infinity Cache between launches)
# under one FETCH_SIZE pass and one WRITE_SIZE pass; the summary sets FETCH_SIZE (raw, and x2) and
# WRITE_SIZE beside the bytes the launch must move: the operand columns it reads (a: N columns, x: K
# columns, each row's contiguous run rounded up to whole 128-byte lines) and the chunk partials it writes.
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_wgrad_calib; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
for shape in "256 256" "129 283" "3 128" "256 63"; do
  set -- $shape
  for c in FETCH_SIZE WRITE_SIZE; do
    N=$1 K=$2 ITERS=4 timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $OUT/n$1k$2_$c -o run --output-format csv \
      -- python3 $ROOT/scripts/wgrad_probe.py > $OUT/n$1k$2_$c.log 2>&1 || { echo "pass $shape $c failed"; tail -3 $OUT/n$1k$2_$c.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, json, collections
out = {}
M, LDA, LDX = 262144, 2312, 2400
def lines(nbytes):           # a row's contiguous run (starting 16-byte aligned) in 128-byte lines
    return -(-nbytes // 128) * 128
for d in sorted(glob.glob('/root/repo/gpurun_out/pmc_wgrad_calib/n*k*_*/run_counter_collection.csv')):
    tag = d.split('/')[-2]
    shape, counter = tag.split('_', 1)
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(d)):
        if 'wgrad' in r['Kernel_Name'] and 'reduce' not in r['Kernel_Name']:
            vals[r['Kernel_Name'].split('(')[0]].append(float(r['Counter_Value']) * 1024)
    for k, v in vals.items():
        out.setdefault(shape, {"kernel": k})[counter] = sum(v[1:]) / max(len(v) - 1, 1)   # first launch: cold
for shape, e in out.items():
    n, k = int(shape[1:shape.index('k')]), int(shape[shape.index('k') + 1:])
    e["read_bytes_lines"] = M * (lines(4 * n) + lines(4 * k))
    e["read_bytes_exact"] = M * 4 * (n + k)
    if "FETCH_SIZE" in e:
        e["fetch_raw_over_lines"] = e["FETCH_SIZE"] / e["read_bytes_lines"]
        e["fetch_x2_over_lines"] = 2 * e["FETCH_SIZE"] / e["read_bytes_lines"]
json.dump(out, open('/root/repo/gpurun_out/pmc_wgrad_calib/summary.json', 'w'), indent=1)
print(json.dumps(out, indent=1))
PY
