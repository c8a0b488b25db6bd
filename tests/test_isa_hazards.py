"""ISA check of the built gfx950 code (CPU test, no GPU): every DPP instruction's source VGPRs must
not have been written by a VALU instruction within the 2 wait states gfx9 requires before a DPP read
(VALU write -> DPP read hazard). The row kernel issues its DPP fmacs from inline asm, which the
compiler's hazard recognizer cannot see into (vecchia_rows16.hip `fmac_bcast16`), so this scans the
shipped library's disassembly instead of trusting the schedule.

The scan is linear over each function's instruction stream (a straight-line approximation: the
kernels' DPP sequences are fully unrolled); `s_nop N` counts as N + 1 wait states.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "gpboost_amd", "lib", "libgpboost_amd.so")
OBJDUMP = "/opt/rocm/llvm/bin/llvm-objdump"

_REG = re.compile(r"^v(\d+)$|^v\[(\d+):(\d+)\]$")


def _vregs(tok: str) -> set[int]:
    m = _REG.match(tok.strip())
    if not m:
        return set()
    if m.group(1) is not None:
        return {int(m.group(1))}
    return set(range(int(m.group(2)), int(m.group(3)) + 1))


def _parse(line: str):
    """(mnemonic, operand tokens) of one disassembled instruction line, or None."""
    code = line.split("//")[0].strip()
    if not code or code.endswith(":") or code.startswith("<"):
        return None
    parts = code.split(None, 1)
    ops = [t.strip() for t in parts[1].split(",")] if len(parts) > 1 else []
    # modifiers after the last operand (row_newbcast:1 row_mask:0xf ...) stay attached: strip them
    if ops:
        ops[-1] = ops[-1].split()[0]
    return parts[0], ops


def _valu_writes(mn: str, ops: list[str]) -> set[int]:
    if not mn.startswith("v_") or mn.startswith(("v_cmp", "v_readlane", "v_readfirstlane")) or not ops:
        return set()
    return _vregs(ops[0])


def scan(text: str) -> tuple[int, list[str]]:
    """Number of DPP instructions checked and the hazards found in a disassembly."""
    window: list[tuple[int, set[int], str]] = []   # (wait states the instruction occupies, VGPRs written, text)
    n_dpp, bad = 0, []
    for line in text.splitlines():
        if line.endswith(">:"):   # a new function
            window.clear()
            continue
        p = _parse(line)
        if p is None:
            continue
        mn, ops = p
        if "_dpp" in mn and len(ops) >= 2:
            n_dpp += 1
            # DPP applies to src0: the first source operand (the accumulator of v_fmac is the destination)
            src = _vregs(ops[1])
            waits = 0
            for ws, writes, txt in reversed(window):
                if waits >= 2:
                    break
                if writes & src:
                    bad.append(f"{txt.strip()}  ->  {line.split('//')[0].strip()}")
                    break
                waits += ws
        if mn == "s_nop":
            ws = int(ops[0], 0) + 1 if ops else 1
        else:
            ws = 1
        window.append((ws, _valu_writes(mn, ops), line))
        if len(window) > 8:
            window.pop(0)
    return n_dpp, bad


def test_scanner_flags_a_hazard():
    hazard = ("<k>:\n v_mul_f64 v[4:5], v[0:1], v[2:3]\n"
              " v_fmac_f64_dpp v[8:9], v[4:5], v[6:7] row_newbcast:1 row_mask:0xf bank_mask:0xf\n")
    assert scan(hazard)[1]
    safe = ("<k>:\n v_mul_f64 v[4:5], v[0:1], v[2:3]\n s_nop 1\n"
            " v_fmac_f64_dpp v[8:9], v[4:5], v[6:7] row_newbcast:1 row_mask:0xf bank_mask:0xf\n")
    assert scan(safe) == (1, [])
    unrelated = ("<k>:\n v_mul_f64 v[6:7], v[0:1], v[2:3]\n"
                 " v_fmac_f64_dpp v[8:9], v[4:5], v[6:7] row_newbcast:1 row_mask:0xf bank_mask:0xf\n")
    assert scan(unrelated) == (1, [])


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library or llvm-objdump absent")
def test_no_valu_to_dpp_hazard_in_built_library():
    tmp = tempfile.mkdtemp(prefix="gpb_isa_")
    try:
        lib = os.path.join(tmp, "lib.so")
        shutil.copy(LIB, lib)
        subprocess.run([OBJDUMP, "--offloading", lib], cwd=tmp, check=True, capture_output=True)
        total, hazards = 0, []
        for f in sorted(os.listdir(tmp)):
            if not f.endswith("gfx950"):
                continue
            dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", os.path.join(tmp, f)], check=True,
                                 capture_output=True, text=True).stdout
            n, bad = scan(dis)
            total += n
            hazards += bad
        assert total > 1000, f"expected the row kernels' DPP code, found {total} DPP instructions"
        assert not hazards, f"{len(hazards)} VALU-write -> DPP-read hazards, e.g.:\n" + "\n".join(hazards[:10])
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
