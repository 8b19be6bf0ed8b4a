"""Reduced gfx950 disassemblies of the stream kernels for tests/test_check_isa.py (CPU, no hipcc needed).

For each library build given, keeps from `llvm-objdump -d` of its code objects, for the kernels matching
--kernels: the function headers and every instruction check_isa.check_vmcnt looks at (VM ops, LDS-DMA
pieces and their M0 writes, vmcnt waits, s_barrier, branches, s_endpgm) plus every branch target, with
their addresses.  Writes tests/golden/isa/<name>.txt.gz.

  make -C depth-aware-shader-effects-for-nerf_amd ab NAME=extra1 DEFS=-DNERF16_WAIT_EXTRA=1
  python scripts/make_isa_fixtures.py head=depth-aware-shader-effects-for-nerf_amd/libnerfmi.so \
      extra1=depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_extra1.so ...
"""
import argparse
import gzip
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import check_isa  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEEP = re.compile(r"^(global_|buffer_|scratch_|flat_|s_waitcnt|s_barrier|s_c?branch|s_endpgm|s_setpc|s_nop)")


def reduce(text, kernels):
    out, cur, base, lines = [], None, 0, []

    def flush():
        if cur is None or not re.search(kernels, cur):
            return
        targets = set()
        for ln in lines:
            m = re.search(r"<.*\+(0x[0-9a-f]+)>\s*$", ln)
            if m:
                targets.add(base + int(m.group(1), 16))
        out.append(f"{base:016x} <{cur}>:")
        for ln in lines:
            s = ln.strip()
            ins = s.split("//")[0].strip()
            am = re.search(r"//\s*([0-9A-Fa-f]+):", s)
            addr = int(am.group(1), 16) if am else -1
            if KEEP.match(ins) or re.search(r"\bm0\b", ins) or addr in targets:
                out.append(ln.rstrip())
        out.append("")

    for line in text.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.*)>:$", line)
        if m:
            flush()
            cur, base, lines = m.group(2), int(m.group(1), 16), []
            continue
        if cur is not None and "//" in line:
            lines.append(line)
    flush()
    return "\n".join(out) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", default=r"mlp16_kernel<true>|mlp_backward16_bound_kernel")
    ap.add_argument("builds", nargs="+", help="name=path/to/lib.so")
    a = ap.parse_args()
    dst = os.path.join(REPO, "tests", "golden", "isa")
    os.makedirs(dst, exist_ok=True)
    for spec in a.builds:
        name, lib = spec.split("=", 1)
        text = reduce(check_isa.disassemble(lib), a.kernels)
        with gzip.open(os.path.join(dst, f"{name}.txt.gz"), "wt", compresslevel=9) as f:
            f.write(text)
        print(name, len(text.splitlines()), "lines")


if __name__ == "__main__":
    main()
