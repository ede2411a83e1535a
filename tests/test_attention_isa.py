"""Hazard distances of the hand-written MFMAs in the built code object.

attention_bwd_pipe.hip issues its dK / dV (and dQ) accumulate MFMAs from inline asm, which the
compiler's hazard recognizer does not see.  A VALU instruction that writes a VGPR read by a
following MFMA as SrcA / SrcB needs at least two wait states in between on gfx950; the kernel's
schedule keeps every bf16-packed operand at least two gaps ahead, with no s_nop.  This test
disassembles the gfx950 code object of the built library (tools/isa_dump.py, CPU only) and checks,
for every asm MFMA (the ones accumulating into AGPRs), the distance to the nearest VALU writer of
its source registers within the basic block.
"""
import re
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))

MIN_WAIT_STATES = 2


def _regs(op: str):
    m = re.fullmatch(r"v(\d+)", op)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def _split(line: str):
    parts = line.split(None, 1)
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    return parts[0], ops


def _valu_dest(mnem: str, ops):
    if not mnem.startswith("v_") or mnem.startswith(("v_cmp", "v_readfirstlane", "v_readlane", "v_mfma")):
        return set()
    return _regs(ops[0]) if ops else set()


def _check(body):
    worst, n_mfma = None, 0
    for idx, line in enumerate(body):
        mnem, ops = _split(line)
        if not mnem.startswith("v_mfma") or not ops or not ops[0].startswith("a["):
            continue
        n_mfma += 1
        srcs = _regs(ops[1]) | _regs(ops[2])
        waits = 0
        for back in range(idx - 1, -1, -1):
            m2, o2 = _split(body[back])
            if m2.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm")):
                break
            if _valu_dest(m2, o2) & srcs:
                worst = waits if worst is None else min(worst, waits)
                break
            waits += (int(o2[0]) + 1) if m2 == "s_nop" and o2 else 1
    return worst, n_mfma


@pytest.mark.parametrize("kernel", ["attn_bwd_dkdv_pipe_kernel", "attn_bwd_dq_pipe_kernel"])
def test_asm_mfma_operands_are_two_wait_states_after_their_valu_writers(kernel):
    import isa_dump
    lib = ROOT / "pytorch_operator_amd" / "_lib" / "libpto_hip.so"
    if not lib.exists():
        from pytorch_operator_amd.ops import _native
        _native.build()
    bodies = isa_dump.kernel_bodies(isa_dump.disassemble(lib), kernel)
    assert bodies, f"{kernel} not found in the code object"
    for sym, body in bodies.items():  # every instantiation (the dQ pass has 8- and 4-wave ones)
        worst, n = _check(body)
        assert n > 0, (sym, "no hand-written (AGPR-accumulating) MFMA found")
        assert worst is None or worst >= MIN_WAIT_STATES, (sym, worst)


def test_checker_flags_a_too_close_writer():
    body = ["v_cvt_pk_bf16_f32 v20, v1, v2", "v_add_f32_e32 v3, v4, v5",
            "v_mfma_f32_32x32x16_bf16 a[0:15], v[20:23], v[24:27], a[0:15]"]
    assert _check(body) == (1, 1)
    body.insert(2, "s_nop 0")
    assert _check(body) == (2, 1)
