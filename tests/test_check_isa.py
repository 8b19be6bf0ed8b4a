"""The build-time M0 guard (scripts/check_isa.py, `make check-isa`): the LDS-DMA weight streams of
mlp16_kernel and mlp_backward16_lds_kernel declare M0 clobbered, so nothing else in those kernels may
read M0.  The check passes on the shipped libnerfmi.so and fails on the same disassembly with an M0
reader inserted (explicit operand, implicit reader, a write the DMA does not consume)."""
import os
import re
import shutil
import sys

import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "scripts"))
import check_isa  # noqa: E402

LIB = os.path.join(REPO, "depth-aware-shader-effects-for-nerf_amd", "libnerfmi.so")
pytestmark = pytest.mark.skipif(not (os.path.exists(LIB) and shutil.which(os.path.join(check_isa.LLVM, "llvm-objdump"))),
                                reason="needs the built library and ROCm's llvm-objdump")


@pytest.fixture(scope="module")
def disasm():
    return check_isa.disassemble(LIB)


def test_shipped_library_is_clean(disasm):
    report, checked = check_isa.check(disasm)
    assert any("mlp16_kernel<false>" in n for n in checked) and any("mlp16_kernel<true>" in n for n in checked)
    assert any("mlp_backward16_lds_kernel" in n for n in checked)
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


@pytest.mark.parametrize("kernel", ["mlp16_kernel<false>", "mlp_backward16_lds_kernel"])
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
