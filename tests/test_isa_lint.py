"""MFMA hazard lint (tools/isa_lint.py) over the built matrix-core kernels, on the CPU.

Round 1 saw stale MFMA sums when a read of the accumulators sat after a branch
("MFMA hazard").  gfx950 does not interlock a VALU access to an XDL
result: the compiler pads straight-line code with s_nop.  The lint walks every
control-flow path out of every MFMA in the built code object and fails when one
reaches an access to the MFMA's destination registers in fewer wait states than
the op needs, so an edit that moves a read behind a branch fails here, before
any GPU run."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_lint  # noqa: E402

OBJ = os.path.join(ROOT, "find-tfbs_amd", "lib", "obj", "scan_mfma.o")


def test_built_mfma_kernels_respect_wait_states():
    assert os.path.exists(OBJ), "build first (make)"
    text = isa_lint.disassemble(OBJ)
    n_mfma = sum(1 for line in text.splitlines() if "v_mfma_scale_f32_32x32x64_f8f6f4" in line)
    assert n_mfma >= 16  # every depth variant's MFMAs are there
    assert isa_lint.lint_text(text) == []


_F = "0000000000001000 <k>:\n"


def _insn(addr, text, target=""):
    return "\t%-50s // %012X: 00000000%s\n" % (text, addr, (" <k+0x%x>" % target) if target else "")


def test_lint_flags_short_straight_line_path():
    text = _F + _insn(0x1000, "v_mfma_scale_f32_32x32x64_f8f6f4 v[2:17], v[20:23], v[24:29], 0, v30, v30") + \
        _insn(0x1010, "s_nop 3") + _insn(0x1014, "v_max_f32_e32 v1, v2, v3") + _insn(0x1018, "s_endpgm")
    bad = isa_lint.lint_text(text)
    assert len(bad) == 1 and "4 wait states" in bad[0]
    ok = _F + _insn(0x1000, "v_mfma_scale_f32_32x32x64_f8f6f4 v[2:17], v[20:23], v[24:29], 0, v30, v30") + \
        _insn(0x1010, "s_nop 11") + _insn(0x1014, "v_max_f32_e32 v1, v2, v3") + _insn(0x1018, "s_endpgm")
    assert isa_lint.lint_text(ok) == []


def test_lint_follows_branches():
    """The padding before the branch is enough on the fall-through path but the
    branch target reads the accumulators right away."""
    text = _F + _insn(0x1000, "v_mfma_scale_f32_32x32x64_f8f6f4 v[2:17], v[20:23], v[24:29], 0, v30, v30") + \
        _insn(0x1010, "s_cbranch_scc1 3", 0x20) + _insn(0x1014, "s_nop 11") + \
        _insn(0x1018, "v_max_f32_e32 v1, v2, v3") + _insn(0x101c, "s_endpgm") + \
        _insn(0x1020, "v_max_f32_e32 v1, v16, v17") + _insn(0x1024, "s_endpgm")
    bad = isa_lint.lint_text(text)
    assert len(bad) == 1 and "+0x20" in bad[0]
