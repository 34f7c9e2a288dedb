#!/usr/bin/env python3
"""MFMA result hazard lint over a built gfx950 code object.

A VALU (or any non-MFMA) instruction that reads or writes a VGPR an XDL MFMA
wrote must issue at least N wait states after it (each instruction counts one,
`s_nop k` counts k + 1); gfx950 does not interlock these.  The compiler pads
straight-line code itself; round 1 saw stale MFMA sums when a read sat after a
branch (MFMA hazard).  This lint walks every path out of every MFMA
(fall-through and branch targets) and reports any access to its destination
registers before N wait states.

N = 12 for v_mfma_scale_f32_32x32x64_f8f6f4 (an 8-pass XDL op on gfx950; the
compiler's own straight-line padding of it is s_nop 11 after a lone MFMA).

Usage: python tools/isa_lint.py OBJECT.o   (the host object hipcc built; its
.hip_fatbin bundle is unpacked with clang-offload-bundler and disassembled with
llvm-objdump)
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REQUIRED = {"v_mfma_scale_f32_32x32x64_f8f6f4": 12}
DEFAULT_REQUIRED = 19  # any other MFMA: the 16-pass XDL figure, the largest

_INSN = re.compile(r"^\s+([a-z_0-9]+)(.*?)\s*//\s*([0-9A-Fa-f]+):")
_FUNC = re.compile(r"^([0-9a-fA-F]+) <(.+)>:$")
_TARGET = re.compile(r"<(.+)\+0x([0-9a-fA-F]+)>\s*$")
_VREG = re.compile(r"\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]")  # VGPRs and AGPRs (AGPR a_i -> 1024 + i)


def disassemble(obj):
    """-> llvm-objdump text of the gfx950 code object inside a hipcc object file."""
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin")
        subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fb, obj,
                               os.path.join(d, "x.o")])
        co = os.path.join(d, "k.co")
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                               "--input=" + fb, "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co])
        return subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co],
                                       text=True)


def regs(operands):
    out = set()
    for m in _VREG.finditer(operands):
        if m.group(1) is not None:
            out.add(int(m.group(2)) + (1024 if m.group(1) == "a" else 0))
        else:
            b = 1024 if m.group(3) == "a" else 0
            out.update(range(b + int(m.group(4)), b + int(m.group(5)) + 1))
    return out


def parse(text):
    """-> {function: [(addr, mnemonic, operands, line)]}"""
    funcs, cur = {}, None
    for line in text.splitlines():
        f = _FUNC.match(line)
        if f:
            cur = funcs.setdefault(f.group(2), [])
            continue
        m = _INSN.match(line)
        if m and cur is not None:
            cur.append((int(m.group(3), 16), m.group(1), m.group(2), line))
    return funcs


def lint_function(name, insns):
    """-> list of violations (text)"""
    if not insns:
        return []
    base = insns[0][0]
    at = {a: i for i, (a, _, _, _) in enumerate(insns)}
    succ = []
    for i, (a, mn, ops, line) in enumerate(insns):
        nxt = [i + 1] if i + 1 < len(insns) else []
        if mn == "s_endpgm" or mn.startswith("s_setpc") or mn.startswith("s_swappc"):
            nxt = []
        elif mn.startswith("s_branch") or mn.startswith("s_cbranch"):
            t = _TARGET.search(line)
            tgt = at.get(base + int(t.group(2), 16)) if t else None
            if tgt is None:
                raise ValueError("%s: unresolved branch at %x" % (name, a))
            nxt = [tgt] if mn.startswith("s_branch") else nxt + [tgt]
        succ.append(nxt)

    def cost(i):
        mn, ops = insns[i][1], insns[i][2]
        if mn == "s_nop":
            return int(ops.strip().split()[0], 0) + 1
        return 1

    bad = []
    for i, (a, mn, ops, line) in enumerate(insns):
        if not mn.startswith("v_mfma"):
            continue
        need = REQUIRED.get(mn, DEFAULT_REQUIRED)
        dst = regs(ops.split(",")[0])
        best = {}  # fewest wait states with which an instruction can issue after this MFMA
        stack = [(j, 0) for j in succ[i]]
        while stack:
            j, ws = stack.pop()
            if ws >= need or best.get(j, need) <= ws:
                continue
            best[j] = ws
            mnj, opsj = insns[j][1], insns[j][2]
            hit = regs(opsj) & dst
            if not mnj.startswith("v_mfma") and hit:
                bad.append("%s+0x%x: %s%s touches register %d %d wait states after the MFMA at +0x%x (needs %d)" % (
                    name[:60], insns[j][0] - base, mnj, opsj.rstrip()[:40], min(hit), ws, a - base, need))
                continue
            for k in succ[j]:
                stack.append((k, ws + cost(j)))
    return bad


def lint_text(text):
    out = []
    for name, insns in parse(text).items():
        out += lint_function(name, insns)
    return out


def main():
    text = disassemble(sys.argv[1])
    n = sum(1 for line in text.splitlines() if "v_mfma" in line)
    bad = lint_text(text)
    for b in bad:
        print(b)
    print("%d MFMAs checked, %d violations" % (n, len(bad)))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
