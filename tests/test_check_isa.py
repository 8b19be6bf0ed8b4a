"""The build-time ISA guard (scripts/check_isa.py, `make check-isa`, run by __graft_entry__.build()).

M0: the LDS-DMA weight streams of mlp16_kernel and mlp_backward16_bound_kernel declare M0 clobbered, so
nothing else in those kernels may read M0.  The check passes on the shipped libnerfmi.so and fails on
the same disassembly with an M0 reader inserted (explicit operand, implicit reader, a write the DMA does
not consume).

vmcnt: every publish of an LDS-DMA ring (the counted `s_waitcnt vmcnt(N)` + `s_barrier` of
stream16.h, shared by the forward and the data gradient) must leave in flight only pieces younger
than the published chunk, on every path of the kernel's control-flow graph.  Shown on the shipped
library (passes), on the shipped disassembly with one publish over-counted, a flat op in the window
or the exit drain removed (fails), and on committed disassemblies of three builds
(tests/golden/isa, scripts/make_isa_fixtures.py): the default, round 3's store-slack count (passes:
within the window) and NERF16_WAIT_EXTRA=1 (fails at the group-boundary publishes).  On the GPU the
passing builds train bit-identically to each other and the failing ones differ from run to run
(profiles/r04/vmcnt_ab_overcount.log, scripts/vmcnt_ab.py): the check's boundary is the hardware's.

Store data: no instruction may write a data register of a 12- or 16-byte store within 2 wait states of
it (round 6: an unpadded VALU write behind a store with a register soffset changed saved activations
from run to run; csrc/common.h store16_rows).  Shown on hand-written sequences, including the
measured one, and on the shipped training forward with such a write inserted."""
import gzip
import os
import re
import shutil
import sys

import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "scripts"))
import check_isa  # noqa: E402

LIB = os.path.join(REPO, "depth-aware-shader-effects-for-nerf_amd", "libnerfmi.so")
ISA_FIXTURES = os.path.join(REPO, "tests", "golden", "isa")


@pytest.mark.parametrize("build,ok", [("head", True), ("r3slack", True), ("extra1", False)])
def test_vmcnt_on_committed_builds(build, ok):
    text = gzip.open(os.path.join(ISA_FIXTURES, f"{build}.txt.gz"), "rt").read()
    report, checked = check_isa.check(text)
    assert len(checked) == 2          # mlp16_kernel<true>, mlp_backward16_bound_kernel
    if ok:
        assert report == {}, report
    else:
        assert set(report) == set(checked), report
        assert all(all("publishes" in b for b in v) for v in report.values()), report


def _toy_kernel(n_loop_wait, n_pro_wait=4, drain=True):
    """A hand-written stream kernel: chunks 0 and 1 (4 pieces each), publish 0, then a loop whose every
    iteration issues the next chunk, stores (or not: a branch skips the store) and publishes."""
    a = iter(range(0x100, 0x1000, 4))
    L = ["0000000000000100 <k>:"]

    def ins(t, tgt=None):
        x = next(a)
        L.append(f"\t{t} // {x:012X}: 0" + (f" <k+0x{tgt - 0x100:x}>" if tgt is not None else ""))
        return x
    for _ in range(8):
        ins("s_mov_b32 m0, s4"); ins("global_load_lds_dwordx4 v1, s[2:3]")
    ins(f"s_waitcnt vmcnt({n_pro_wait})"); ins("s_barrier")
    top = ins("s_add_u32 s6, s6, 1")
    for _ in range(4):
        ins("s_mov_b32 m0, s4"); ins("global_load_lds_dwordx4 v1, s[2:3]")
    L.append(None); br, bra = len(L) - 1, next(a)      # s_cbranch_execz over the store
    ins("buffer_store_dword v2, v3, s[8:11], 0 offen")
    join = ins("s_nop 0")
    L[br] = f"\ts_cbranch_execz 1 // {bra:012X}: 0 <k+0x{join - 0x100:x}>"
    ins(f"s_waitcnt vmcnt({n_loop_wait})"); ins("s_barrier")
    ins("s_cbranch_scc1 0", tgt=top)
    if drain:
        ins("s_waitcnt vmcnt(0)")
    ins("s_endpgm")
    return check_isa._instructions("\n".join(L))["k"]


def test_vmcnt_cfg_model():
    """The toy kernel's exact counts pass; one more in the loop (the path that skips the store leaves
    only the 4 pieces younger than the published chunk) or in the prologue is caught, and so is an
    exit without the drain."""
    assert check_isa.check_vmcnt(_toy_kernel(4), 4) == []
    assert check_isa.check_vmcnt(_toy_kernel(5), 4)
    assert check_isa.check_vmcnt(_toy_kernel(4, n_pro_wait=5), 4)
    assert any("ends" in b for b in check_isa.check_vmcnt(_toy_kernel(4, drain=False), 4))


@pytest.fixture(scope="module")
def disasm():
    if not (os.path.exists(LIB) and shutil.which(os.path.join(check_isa.LLVM, "llvm-objdump"))):
        pytest.skip("needs the built library and ROCm's llvm-objdump")
    return check_isa.disassemble(LIB)


def test_shipped_library_is_clean(disasm):
    report, checked = check_isa.check(disasm)
    assert any("mlp16s_kernel" in n for n in checked) and any("mlp16_kernel<true>" in n for n in checked)
    assert any("mlp_backward16_bound_kernel" in n for n in checked)
    assert report == {}, report


def _insert(text, kernel, line, after=5):
    """Insert an instruction line `after` instructions into the first function matching `kernel`."""
    out, state, n = [], 0, 0
    for ln in text.splitlines():
        out.append(ln)
        if state == 0 and re.match(r"^[0-9a-f]+ <.*" + re.escape(kernel) + r".*>:$", ln):
            state = 1
        elif state == 1 and ln.startswith("\t") and ln.strip():
            n += 1
            if n == after:
                out.append("\t" + line)
                state = 2
    assert state == 2
    return "\n".join(out)


@pytest.mark.parametrize("kernel", ["mlp16s_kernel", "mlp_backward16_bound_kernel"])
@pytest.mark.parametrize("line", ["s_movrel_b32 s0, s1", "ds_read_addtid_b32 v0", "s_mov_b32 s3, m0",
                                  "s_mov_b32 m0, 0x100", "v_readfirstlane_b32 s2, v1 ; s_add_u32 s2, s2, m0"])
def test_inserted_m0_reader_is_caught(disasm, kernel, line):
    report, _ = check_isa.check(_insert(disasm, kernel, line))
    assert any(kernel in n for n in report), line


def test_unconsumed_m0_write_is_caught(disasm):
    # a DMA piece whose M0 write is followed by another instruction before the load
    lines = disasm.splitlines()
    for i, ln in enumerate(lines):
        if re.search(r"s_mov_b32 m0, s\d+", ln) and "global_load_lds" in lines[i + 2]:
            lines.insert(i + 1, "\tv_mov_b32_e32 v0, 0")
            break
    report, _ = check_isa.check("\n".join(lines))
    assert report


# ---- counted vmcnt waits of the LDS-DMA streams (check_isa.check_vmcnt) ---------------------------
def test_stream_kernels_are_checked(disasm):
    report, checked = check_isa.check(disasm)
    for k in ("mlp16_kernel<true>", "mlp16s_kernel", "mlp_backward16_bound_kernel"):
        assert any(k in n for n in checked), k
    assert report == {}, report


def _publish_waits(text, kernel):
    """Line indices of the counted waits (vmcnt(N), N > 0) that directly precede an s_barrier in `kernel`."""
    lines = text.splitlines()
    inside, out = False, []
    for i, ln in enumerate(lines):
        if re.match(r"^[0-9a-f]+ <.*>:$", ln):
            inside = kernel in ln
            continue
        if inside and re.search(r"s_waitcnt vmcnt\(([1-9]\d*)\)", ln):
            for x in lines[i + 1:i + 12]:            # the next barrier, before any other vmcnt wait
                if "vmcnt" in x or re.match(r"^[0-9a-f]+ <", x):
                    break
                if "s_barrier" in x:
                    out.append(i)
                    break
    return lines, out


@pytest.mark.parametrize("kernel", ["mlp16_kernel<true>", "mlp_backward16_bound_kernel"])
def test_overcounted_publish_wait_is_caught(disasm, kernel):
    """One publish wait counting one op more than issued after its chunk's pieces, in the ISA text."""
    lines, waits = _publish_waits(disasm, kernel)
    assert waits
    i = waits[len(waits) // 2]
    lines[i] = re.sub(r"vmcnt\((\d+)\)", lambda m: f"vmcnt({int(m.group(1)) + 8})", lines[i])
    report, _ = check_isa.check("\n".join(lines))
    assert any(kernel in n and any("publishes" in b for b in v) for n, v in report.items()), report


def test_flat_op_in_flight_window_is_caught(disasm):
    lines = disasm.splitlines()
    inside = False
    for i, ln in enumerate(lines):
        if re.match(r"^[0-9a-f]+ <.*>:$", ln):
            inside = "mlp16_kernel<true>" in ln
        elif inside and "global_load_lds_dwordx4" in ln:
            addr = re.search(r"//\s*([0-9A-F]+):", ln).group(1)
            lines.insert(i + 1, f"\tflat_store_dword v[0:1], v2 // {addr}: 00000000")
            break
    report, _ = check_isa.check("\n".join(lines))
    assert any("mlp16_kernel<true>" in n and any("flat op" in b for b in v) for n, v in report.items()), report


# ---- store-data wait states (check_isa.check_store_data) -----------------------------------------
@pytest.mark.parametrize("insns,n_bad", [
    # the round-6 failure (training forward, scripts/diag_train_det.py): the first data VGPR of a
    # 16-byte store with a register soffset overwritten by the next instruction
    (["buffer_store_dwordx4 v[6:9], v20, s[24:27], s60 offen nt", "v_accvgpr_read_b32 v6, a84"], 1),
    (["buffer_store_dwordx4 v[6:9], v20, s[24:27], 0 offen nt", "s_nop 1", "v_accvgpr_read_b32 v6, a84"], 0),
    (["buffer_store_dwordx4 v[6:9], v20, s[24:27], 0 offen nt", "s_nop 0", "v_fma_f32 v9, v1, v2, v3"], 1),
    (["buffer_store_dwordx4 v[6:9], v20, s[24:27], 0 offen nt", "v_mfma_f32_32x32x16_f16 a[0:15], v[0:3], v[4:7], a[0:15]",
      "ds_read_b32 v8, v235"], 1),
    (["buffer_store_dwordx4 v[6:9], v20, s[24:27], 0 offen nt", "v_add_u32_e32 v10, 1, v6", "v_mov_b32_e32 v11, 0",
      "v_mov_b32_e32 v6, 0"], 0),                               # (reads, other registers, then 2 states passed)
    (["buffer_store_dword v6, v20, s[24:27], 0 offen", "v_mov_b32_e32 v6, 0"], 0),   # 4-byte store: no hazard
    (["global_store_dwordx4 v[0:1], v[6:9], off", "v_mov_b32_e32 v7, 0"], 1),
])
def test_store_data_rule(insns, n_bad):
    assert len(check_isa.check_store_data(insns)) == n_bad, insns


def test_store_data_overwrite_in_shipped_kernel_is_caught(disasm):
    """The shipped training forward with a VALU write of a store's first data VGPR inserted right behind
    it fails; with two wait states before that write it passes again."""
    lines = disasm.splitlines()
    inside = False
    for i, ln in enumerate(lines):
        if re.match(r"^[0-9a-f]+ <.*>:$", ln):
            inside = "mlp16_kernel<true>" in ln
        elif inside and "buffer_store_dwordx4" in ln:
            first = re.search(r"buffer_store_dwordx4\s+v\[(\d+):", ln).group(1)
            break
    bad = lines[:i + 1] + [f"\tv_mov_b32_e32 v{first}, 0"] + lines[i + 1:]
    report, _ = check_isa.check("\n".join(bad))
    assert any("mlp16_kernel<true>" in n and any("wait state" in b for b in v) for n, v in report.items()), report
    padded = lines[:i + 1] + ["\ts_nop 1", f"\tv_mov_b32_e32 v{first}, 0"] + lines[i + 1:]
    report, _ = check_isa.check("\n".join(padded))
    assert report == {}, report
