"""Build-time guard of the M0 register in the LDS-DMA weight streams (csrc/mlp16.hip, csrc/train.hip).

The streams issue `s_mov_b32 m0, <lds address>` + `global_load_lds_dwordx4` from inline asm and declare
M0 clobbered; the compiler is never told the value must survive, so the kernels are only correct
while no other instruction in them reads M0.  This script disassembles the gfx950 code objects
inside libnerfmi.so (the shipped library: its .hip_fatbin section, one clang offload bundle per
translation unit) and checks, in every kernel whose name matches --kernels:

  * every instruction that writes M0 is `s_mov_b32 m0, s<n>` immediately followed (s_nop aside)
    by the LDS-DMA load that consumes it, or is the restore of a saved piece
    (`s_mov_b32 s<k>, m0; s_mov_b32 m0, s<n>; [s_nop]; <LDS-DMA>; s_mov_b32 m0, s<k>`: the per-ray
    feature-row DMA of mlp16.hip, which saves M0 instead of clobbering it);
  * no other instruction names M0 as an operand or reads it implicitly (s_movrel*, v_movrel*,
    s_set_gpr_idx*, ds_*_addtid*, ds_gws_*, ds_append/ds_consume, ds_ordered_count, s_sendmsg*,
    v_interp*, and any LDS-DMA load that is not directly behind its own M0 write);
  * the stream kernels (--streams) hold at least one DMA piece (the pattern is still what the
    stream emits).

Exit status 0 = clean; 1 = a violation (listed).  `make check-isa` runs it; tests/test_check_isa.py
runs it on the built library and on a disassembly with an M0 reader inserted.
"""
import argparse
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
DEFAULT_KERNELS = r"mlp16_kernel|mlp_backward16|wgrad_dma256"
DEFAULT_STREAMS = r"mlp16_kernel|mlp_backward16_lds|mlp_backward16_bound|wgrad_dma256"
IMPLICIT_M0 = re.compile(r"^(s_movrel|v_movrel|s_set_gpr_idx|ds_\w*addtid|ds_gws_|ds_append|ds_consume|"
                         r"ds_ordered_count|s_sendmsg|v_interp|s_ttracedata)")
LDS_DMA = re.compile(r"^(global_load_lds_|buffer_load_\w+.*\blds\b|buffer_load_lds_)")
M0_OPERAND = re.compile(r"(?<![\w.])m0(?![\w.])")


def code_objects(lib, arch):
    """gfx950 code objects (bytes) of every offload bundle in the library's .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as tmp:
        fat = os.path.join(tmp, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", lib],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
    out = []
    for m in re.finditer(re.escape(MAGIC), data):
        base = m.start()
        (n,) = struct.unpack_from("<Q", data, base + 24)
        at = base + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, at)
            triple = data[at + 24: at + 24 + tlen].decode()
            at += 24 + tlen
            if triple.endswith(arch) or triple.endswith(arch + "-"):
                out.append(data[base + off: base + off + size])
    return out


def disassemble(lib, arch="gfx950"):
    texts = []
    with tempfile.TemporaryDirectory() as tmp:
        for i, co in enumerate(code_objects(lib, arch)):
            path = os.path.join(tmp, f"co{i}.o")
            open(path, "wb").write(co)
            r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "-C", "--no-show-raw-insn",
                                f"--mcpu={arch}", path], check=True, capture_output=True, text=True)
            texts.append(r.stdout)
    return "\n".join(texts)


def functions(text):
    """{demangled name: [instruction lines]} from llvm-objdump -d -C output."""
    funcs, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        s = line.strip()
        if not s or s.startswith(";") or s.endswith(":"):
            continue
        s = s.split("//")[0].strip()
        if s:
            funcs[cur].append(s)
    return funcs


def check_function(insns):
    """Violations in one kernel's instruction list, and its DMA-piece count."""
    bad, pieces = [], 0
    pending = None                     # index of an M0 write waiting for its DMA
    real = [(i, ins) for i, ins in enumerate(insns) if ins.split()[0] != "s_nop"]
    j = 0
    while j < len(real):
        i, ins = real[j]
        op = ins.split()[0]
        operands = ins[len(op):]
        # a saved piece: s_mov_b32 sK, m0 ; s_mov_b32 m0, sN ; DMA ; s_mov_b32 m0, sK
        save = re.match(r"^\s*(s\d+)\s*,\s*m0\s*$", operands) if op == "s_mov_b32" else None
        if save and j + 3 < len(real):
            k = save.group(1)
            w, dma, rest = real[j + 1][1], real[j + 2][1], real[j + 3][1]
            if (re.match(r"^s_mov_b32\s+m0\s*,\s*s\d+\s*$", w) and LDS_DMA.match(dma)
                    and re.match(rf"^s_mov_b32\s+m0\s*,\s*{k}\s*$", rest) and pending is None):
                pieces += 1
                j += 4
                continue
        j += 1
        if LDS_DMA.match(ins):
            if pending is None:
                bad.append(f"{i}: LDS-DMA load not directly behind its own M0 write: {ins}")
            else:
                pieces += 1
            pending = None
            continue
        if pending is not None:
            bad.append(f"{pending}: M0 written but not consumed by the next instruction ({ins})")
            pending = None
        writes_m0 = re.match(r"^\s*m0\s*,", operands) is not None
        if writes_m0:
            if op == "s_mov_b32" and re.match(r"^\s*m0\s*,\s*s\d+\s*$", operands):
                pending = i
            else:
                bad.append(f"{i}: M0 written by something other than a DMA piece: {ins}")
            continue
        if M0_OPERAND.search(operands):
            bad.append(f"{i}: reads M0: {ins}")
        elif IMPLICIT_M0.match(op):
            bad.append(f"{i}: reads M0 implicitly: {ins}")
    if pending is not None:
        bad.append(f"{pending}: M0 written at the end of the kernel without a DMA")
    return bad, pieces


def check(text, kernels=DEFAULT_KERNELS, streams=DEFAULT_STREAMS):
    """{kernel: violations} over the kernels matching `kernels` (regex), and the checked names."""
    report, checked = {}, []
    for name, insns in functions(text).items():
        if not re.search(kernels, name):
            continue
        checked.append(name)
        bad, pieces = check_function(insns)
        if pieces == 0 and re.search(streams, name):
            bad.append("no LDS-DMA piece found (the stream pattern changed: update this check)")
        if bad:
            report[name] = bad
    return report, checked


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "depth-aware-shader-effects-for-nerf_amd", "libnerfmi.so"))
    ap.add_argument("--kernels", default=DEFAULT_KERNELS)
    ap.add_argument("--arch", default="gfx950")
    a = ap.parse_args()
    report, checked = check(disassemble(a.lib, a.arch), a.kernels)
    if not checked:
        print(f"check_isa: no kernel matching {a.kernels!r} in {a.lib}")
        return 1
    for name in checked:
        print(f"check_isa: {'FAIL' if name in report else 'ok  '} {name}")
        for b in report.get(name, [])[:20]:
            print(f"    {b}")
    return 1 if report else 0


if __name__ == "__main__":
    sys.exit(main())
