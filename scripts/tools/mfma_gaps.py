"""Instruction mix between consecutive MFMAs in a range of an assembly listing (.s from
hipcc -S): prints one line per MFMA gap with the classes issued in it, then totals.
    python scripts/tools/mfma_gaps.py file.s START_LINE END_LINE [--verbose]"""
import re
import sys
from collections import Counter


def cls(op):
    if op.startswith("v_mfma"):
        return "MFMA"
    if op.startswith("v_accvgpr_read"):
        return "AccRd"
    if op.startswith("v_accvgpr_write"):
        return "AccWr"
    if op.startswith("v_accvgpr_mov"):
        return "AccMov"
    if op.startswith("ds_read"):
        return "DSR"
    if op.startswith("ds_write"):
        return "DSW"
    if op.startswith("global_load_lds") or op.startswith("buffer_load") and "lds" in op:
        return "DMA"
    if op.startswith("global_load") or op.startswith("buffer_load") or op.startswith("scratch_load"):
        return "VMEM_R"
    if op.startswith("global_store") or op.startswith("scratch_store") or op.startswith("buffer_store"):
        return "VMEM_W"
    if op.startswith("s_waitcnt"):
        return "WAIT"
    if op.startswith("s_nop"):
        return "NOP"
    if op.startswith("s_barrier"):
        return "BAR"
    if op.startswith("v_cvt"):
        return "CVT"
    if op.startswith("v_"):
        return "VALU"
    if op.startswith("s_"):
        return "SALU"
    return "other"


def main():
    path, a, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    verbose = "--verbose" in sys.argv
    lines = open(path).read().split("\n")[a - 1:b]
    gaps, cur, tot = [], Counter(), Counter()
    for ln in lines:
        s = ln.strip()
        if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        c = cls(op)
        tot[c] += 1
        if c == "MFMA":
            gaps.append(cur)
            cur = Counter()
        else:
            cur[c] += 1
    gaps.append(cur)
    if verbose:
        for i, g in enumerate(gaps):
            print(i, dict(g))
    print("totals", dict(tot))
    # VALU-ish issue slots per gap histogram
    h = Counter(sum(v for k, v in g.items() if k in ("VALU", "CVT", "AccRd", "AccWr", "AccMov")) for g in gaps)
    print("VALU-class per gap histogram", sorted(h.items()))


if __name__ == "__main__":
    main()
