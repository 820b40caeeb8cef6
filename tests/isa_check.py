"""Static checks of libfdfs_gpu's shipped gfx950 code objects (CPU only).

hipcc treats an inline `asm` statement as one opaque instruction: it pads no
wait states inside it and none for a hazard whose producer or consumer sits
inside it (/opt/skills/guides/cdna_hip_programming.md, section 5.7 item 2).
sig_hash_kernel relies on two such hand-managed facts:

* its polynomial MFMA accumulators live in AGPRs -- with VGPR accumulators
  the asm VALU blocks could be allocated onto registers an in-flight MFMA
  still reads or writes (measured wrong planes in fixed lanes, round 2);
* the `s_nop`s in quad_transpose cover the VALU-write -> DPP-read hazard of
  its v_cndmask_b32_dpp butterflies.

This module disassembles the code objects embedded in the built library
(llvm-objdump --offloading, then -d --mcpu=gfx950) and checks both facts
and, generally, every DPP read and every MFMA operand read against the VALU
writes before it, in straight-line instruction order.  A compiler or
register-allocation change that breaks them then fails the CPU test suite
instead of corrupting signatures silently.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import tempfile

LLVM_BIN = "/opt/rocm/lib/llvm/bin"
OBJDUMP = os.path.join(LLVM_BIN, "llvm-objdump")

# Wait states required between a VALU write of a VGPR and a read of it:
# by DPP (src0 read through the DPP network) and by an MFMA (SrcA/B/C):
# 2 each on gfx940/gfx950 (the `s_nop 1` quad_transpose carries).
VALU_TO_DPP = 2
VALU_TO_MFMA = 2

_REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def code_objects(lib_path: str, workdir: str) -> list[str]:
    """The gfx950 code objects of the library's offload bundles (extracted
    into workdir: llvm-objdump writes them next to its input)."""
    local = os.path.join(workdir, os.path.basename(lib_path))
    shutil.copyfile(lib_path, local)
    subprocess.run([OBJDUMP, "--offloading", local], check=True, capture_output=True, text=True)
    return sorted(os.path.join(workdir, f) for f in os.listdir(workdir) if f.endswith("--gfx950"))


def disassemble(co: str) -> dict[str, list[str]]:
    """{function symbol: [instruction text]} of one code object."""
    out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", "--no-show-raw-insn", co], check=True,
                         capture_output=True, text=True).stdout
    funcs: dict[str, list[str]] = {}
    cur = None
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        t = line.split("//")[0].strip()
        if t and not t.endswith(":"):
            funcs[cur].append(t)
    return funcs


def regs(op: str) -> set[tuple[str, int]]:
    """Registers named by one operand: v7 -> {(v, 7)}, v[4:7] -> 4 of them."""
    out = set()
    for kind, lo, hi, one in _REG.findall(op):
        if one:
            out.add((kind, int(one)))
        else:
            out.update((kind, r) for r in range(int(lo), int(hi) + 1))
    return out


def operands(inst: str) -> tuple[str, list[str]]:
    parts = inst.split(None, 1)
    mnem = parts[0]
    if len(parts) == 1:
        return mnem, []
    # modifiers (quad_perm:[..], row_mask:.., offset:.., bitop3:..) follow
    # the operands separated by spaces; operands are comma-separated
    ops = [o.strip() for o in re.split(r",(?![^\[]*\])", parts[1])]
    if ops:
        ops[-1] = ops[-1].split(" ")[0]
    return mnem, ops


def is_valu(mnem: str) -> bool:
    return mnem.startswith("v_") and not mnem.startswith(("v_mfma", "v_smfmac"))


def wait_states(inst: str) -> int:
    m = re.match(r"s_nop\s+(\d+)", inst)
    return int(m.group(1)) + 1 if m else 1


def hazards(insts: list[str]) -> list[str]:
    """VALU write -> DPP src0 read and VALU write -> MFMA operand read pairs
    closer than the required wait states, in straight-line order."""
    bad = []
    parsed = [operands(i) for i in insts]
    for k, (mnem, ops) in enumerate(parsed):
        if mnem.endswith("_dpp") and len(ops) >= 2:
            reads, need, what = regs(ops[1]), VALU_TO_DPP, "DPP"
        elif mnem.startswith("v_mfma") and len(ops) >= 4:
            reads = set()
            for o in ops[1:4]:
                reads |= {r for r in regs(o) if r[0] == "v"}
            need, what = VALU_TO_MFMA, "MFMA"
        else:
            continue
        if not reads:
            continue
        states = 0
        for j in range(k - 1, -1, -1):
            pm, pops = parsed[j]
            if pm.startswith("s_branch") or pm.startswith("s_cbranch") or pm.startswith("s_setpc"):
                break
            if is_valu(pm) and pops and regs(pops[0]) & reads:
                bad.append(f"{what} `{insts[k]}` reads a VGPR written {states} wait state(s) after "
                           f"`{insts[j]}` (needs {need})")
                break
            states += wait_states(insts[j])
            if states >= need:
                break
    return bad


def check_library(lib_path: str) -> dict:
    """{"functions": n, "mfma": {kernel: [dst kinds]}, "dpp": {kernel: count},
    "setprio": {kernel: count}, "hazards": [..]}."""
    res = {"names": [], "functions": 0, "mfma": {}, "dpp": {}, "setprio": {}, "hazards": []}
    with tempfile.TemporaryDirectory() as d:
        for co in code_objects(lib_path, d):
            for fn, insts in disassemble(co).items():
                res["functions"] += 1
                res["names"].append(fn)
                kinds = [operands(i)[1][0][0] for i in insts if i.startswith("v_mfma")]
                if kinds:
                    res["mfma"][fn] = kinds
                ndpp = sum(1 for i in insts if i.split(None, 1)[0].endswith("_dpp"))
                if ndpp:
                    res["dpp"][fn] = ndpp
                nprio = sum(1 for i in insts if i.startswith("s_setprio"))
                if nprio:
                    res["setprio"][fn] = nprio
                res["hazards"] += [f"{fn}: {h}" for h in hazards(insts)]
    return res
