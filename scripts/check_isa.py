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

that no instruction overwrites the data registers of a 12- or 16-byte store within 2 wait states of
it (check_store_data), and, in the stream kernels (STREAM_PIECES), that every counted `s_waitcnt vmcnt(N)` publishing an
LDS-DMA ring slot leaves in flight only pieces younger than the published chunk, on every path of the
kernel's control-flow graph (check_vmcnt, below).

Exit status 0 = clean; 1 = a violation (listed).  `make check-isa` and __graft_entry__.build() run it;
tests/test_check_isa.py runs it on the built library, on disassemblies with an M0 reader inserted or a
publish over-counted, and on committed disassemblies of known-good and known-bad builds.
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
DEFAULT_KERNELS = r"mlp16_kernel|mlp16s_kernel|mlp_backward16"
DEFAULT_STREAMS = r"mlp16_kernel|mlp16s_kernel|mlp_backward16_bound"
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


# ---- counted vmcnt waits of the LDS-DMA streams --------------------------------------------------
# A stream kernel publishes ring slots with `s_waitcnt vmcnt(N)` + `s_barrier`: hipcc does not count
# the asm DMA pieces, so N is written by hand as "the pieces and stores issued after the awaited
# ones".  vmcnt retires loads, stores, atomics and LDS-DMA together in issue order (flat_* excepted),
# so the ops that may still be outstanding after vmcnt(N) are the N youngest issued.  The stream
# protocol: the b-th s_barrier after the kernel's first piece publishes the b-th group of P pieces
# (P = this wave's pieces per chunk / stage), so before it every piece of groups 0..b must be done:
#     (pieces possibly outstanding) <= (pieces issued) - P (b + 1).
# check_vmcnt walks the kernel's control-flow graph with the set of possible (issued - P b,
# outstanding-op sequence) states per block and checks that inequality at every barrier, on every
# path; it also rejects a flat_* op while a DMA piece may be outstanding, and a DMA piece still
# possibly outstanding at s_endpgm.  A count one too large (a store counted as younger than the
# awaited pieces that the scheduler placed before them) fails it; counting fewer is always safe.
# The outstanding sequence is kept 63 deep: the counter holds at most 63 ops and issue stalls on a
# full counter, so an op with 63 younger ones has retired.  Instructions whose vmcnt effect is not
# certain are not counted (counting an op that the hardware does not would be the unsafe direction).
STREAM_PIECES = (  # (kernel regex, this wave's pieces per published chunk / stage)
    (r"mlp16_kernel", 4),
    (r"mlp16s_kernel", 4),
    (r"mlp_backward16_bound_kernel", 4),
)
VM_OP = re.compile(r"^(global_|buffer_(load|store|atomic)|scratch_)")
FLAT_OP = re.compile(r"^flat_")
BRANCH = re.compile(r"^s_(c?branch\w*)")
MAX_STATES = 4096          # per block: a blow-up means the states diverge (a loop that gains pieces)


def _instructions(text):
    """{kernel: [(address, instruction, branch target or None)]} from llvm-objdump -d -C output."""
    funcs, cur, base = {}, None, 0
    for line in text.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.*)>:$", line)
        if m:
            cur, base = m.group(2), int(m.group(1), 16)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        s = line.strip()
        if not s or s.startswith(";") or s.endswith(":") or "//" not in s:
            continue
        ins, comment = s.split("//", 1)
        ins = ins.strip()
        am = re.match(r"\s*([0-9A-Fa-f]+):", comment)
        if not ins or not am:
            continue
        tgt = None
        tm = re.search(r"<.*\+(0x[0-9a-f]+)>\s*$", comment)
        if BRANCH.match(ins) and tm:
            tgt = base + int(tm.group(1), 16)
        elif BRANCH.match(ins) and re.search(r"<[^+]*>\s*$", comment):
            tgt = base
        funcs[cur].append((int(am.group(1), 16), ins, tgt))
    return funcs


def _classify(insns):
    """Per instruction: 'P' stream DMA piece, 'F' saved-M0 DMA piece, 'V' other counted VM op,
    'X' flat op, ('W', n) vmcnt wait, 'B' s_barrier, 'E' s_endpgm, or None."""
    kinds = [None] * len(insns)
    real = [k for k, (_, ins, _) in enumerate(insns) if ins.split()[0] != "s_nop"]
    for j, k in enumerate(real):
        ins = insns[k][1]
        op = ins.split()[0]
        if LDS_DMA.match(ins):
            prev2 = insns[real[j - 2]][1] if j >= 2 else ""
            after = insns[real[j + 1]][1] if j + 1 < len(real) else ""
            saved = re.match(r"^s_mov_b32\s+s\d+\s*,\s*m0\s*$", prev2) and re.match(r"^s_mov_b32\s+m0\s*,\s*s\d+\s*$", after)
            kinds[k] = "F" if saved else "P"
        elif VM_OP.match(op):
            kinds[k] = "V"
        elif FLAT_OP.match(op):
            kinds[k] = "X"
        elif op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", ins)
            if m:
                kinds[k] = ("W", int(m.group(1)))
        elif op == "s_barrier":
            kinds[k] = "B"
        elif op == "s_endpgm":
            kinds[k] = "E"
    return kinds


def check_vmcnt(insns, pieces_per_group, margins=None):
    """Violations of the stream protocol (see above) in one kernel: [str].  margins (a dict), if
    given, gets {barrier address: (smallest D - P - outstanding pieces over all states, wait count)}:
    how many more pieces each publish could leave in flight."""
    if not insns:
        return []
    kinds = _classify(insns)
    addr_ix = {a: k for k, (a, _, _) in enumerate(insns)}
    # basic blocks
    leaders = {0}
    for k, (_, ins, tgt) in enumerate(insns):
        if BRANCH.match(ins) or kinds[k] == "E" or ins.startswith("s_setpc"):
            if k + 1 < len(insns):
                leaders.add(k + 1)
            if tgt is not None:
                if tgt not in addr_ix:
                    return [f"{insns[k][0]:x}: branch target {tgt:x} is not an instruction"]
                leaders.add(addr_ix[tgt])
    starts = sorted(leaders)
    block_of = {}
    blocks = []
    for bi, st in enumerate(starts):
        end = starts[bi + 1] if bi + 1 < len(starts) else len(insns)
        blocks.append((st, end))
        block_of[st] = bi
    succ = []
    for st, end in blocks:
        _, ins, tgt = insns[end - 1]
        op = ins.split()[0]
        s = []
        if op == "s_branch":
            s = [block_of[addr_ix[tgt]]]
        elif op.startswith("s_cbranch"):
            s = [block_of[addr_ix[tgt]]] + ([block_of[end]] if end in block_of else [])
        elif op in ("s_endpgm",) or op.startswith("s_setpc"):
            s = []
        elif end in block_of:
            s = [block_of[end]]
        succ.append(s)
    bad = []
    seen = [set() for _ in blocks]
    # state: (started, D = issued pieces - P * publishes, outstanding ops oldest first)
    work = [(0, (False, 0, ()))]
    seen[0].add((False, 0, ()))
    while work:
        bi, state = work.pop()
        started, D, out = state
        last_wait = None
        st, end = blocks[bi]
        for k in range(st, end):
            kd = kinds[k]
            if kd is None:
                continue
            where = f"{insns[k][0]:x}: {insns[k][1]}"
            if kd == "P":
                started, D, out = True, D + 1, (out + ("P",))[-63:]
            elif kd in ("F", "V"):
                out = (out + (kd,))[-63:]
            elif kd == "X":
                if "P" in out or "F" in out:
                    bad.append(f"{where}: flat op while an LDS-DMA piece may be outstanding (flat retires out of order)")
            elif kd[0] == "W":
                n = last_wait = kd[1]
                out = out[-n:] if n else ()
            elif kd == "B" and started:
                w = out.count("P")
                if margins is not None:
                    a = insns[k][0]
                    old = margins.get(a, (1 << 30, None))[0]
                    margins[a] = (min(old, D - pieces_per_group - w), last_wait)
                if w > D - pieces_per_group:
                    bad.append(f"{where}: barrier publishes a group whose pieces may be outstanding "
                               f"({w} pieces may be in flight, at most {D - pieces_per_group} allowed)")
                D -= pieces_per_group
            elif kd == "E":
                if "P" in out or "F" in out:
                    bad.append(f"{where}: kernel ends with an LDS-DMA piece possibly outstanding")
        if abs(D) > 64:
            bad.append(f"{insns[end - 1][0]:x}: pieces issued and published diverge on some path (D = {D})")
            continue
        nxt = (started, D, out)
        for sb in succ[bi]:
            if nxt not in seen[sb]:
                if len(seen[sb]) >= MAX_STATES:
                    bad.append(f"{insns[blocks[sb][0]][0]:x}: too many states (the check does not converge)")
                    return sorted(set(bad))
                seen[sb].add(nxt)
                work.append((sb, nxt))
    return sorted(set(bad))


# ---- store-data wait states ----------------------------------------------------------------------
# A buffer/global store of more than 8 bytes reads its data VGPRs after it issues; an instruction that
# writes one of them too soon can change what is stored.  The compiler models this only for stores
# whose soffset is not a register (csrc/common.h store16_rows), and round 6 measured the unpadded case
# corrupting saved activations in the training forward.  Checked: no instruction within 2 wait states
# after such a store (s_nop N counts N + 1) writes one of its data registers.
WIDE_STORE = re.compile(r"^(buffer_store_dwordx[34]|global_store_dwordx[34]|buffer_store_b(96|128)|"
                        r"global_store_b(96|128))\b")
REG_WRITER = re.compile(r"^(v_|ds_read|ds_load|buffer_load|global_load|scratch_load)")
STORE_DATA_STATES = 2


def _regs(op):
    m = re.match(r"^([va])\[(\d+):(\d+)\]$", op)
    if m:
        return {f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    return {op} if re.match(r"^[va]\d+$", op) else set()


def check_store_data(insns):
    """Violations of the store-data wait states in one kernel's instruction list."""
    bad = []
    for i, ins in enumerate(insns):
        op = ins.split()[0]
        if not WIDE_STORE.match(op):
            continue
        ops = [o.strip() for o in ins[len(op):].split(",")]
        data = _regs(ops[1] if op.startswith("global_") else ops[0])
        states = 0
        for nxt in insns[i + 1:]:
            if states >= STORE_DATA_STATES:
                break
            nop = nxt.split()[0]
            if nop == "s_nop":
                states += int(nxt.split()[1], 0) + 1
                continue
            if REG_WRITER.match(nop) and "_lds" not in nop and _regs(nxt[len(nop):].split(",")[0].strip()) & data:
                bad.append(f"{i}: {ins} -> {nxt} after {states} wait state(s)")
                break
            states += 1
    return bad


def check(text, kernels=DEFAULT_KERNELS, streams=DEFAULT_STREAMS):
    """{kernel: violations} over the kernels matching `kernels` (regex), and the checked names."""
    report, checked = {}, []
    addressed = _instructions(text)
    for name, insns in functions(text).items():
        if not re.search(kernels, name):
            continue
        checked.append(name)
        bad, pieces = check_function(insns)
        bad += check_store_data(insns)
        if pieces == 0 and re.search(streams, name):
            bad.append("no LDS-DMA piece found (the stream pattern changed: update this check)")
        for pat, per in STREAM_PIECES:
            if re.search(pat, name):
                bad += check_vmcnt(addressed.get(name, []), per)
                break
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
