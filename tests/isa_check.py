"""Static checks of libfdfs_gpu's shipped gfx950 code objects (CPU only).

hipcc treats an inline `asm` statement as one opaque instruction: it pads no
wait states inside it and none for a hazard whose producer or consumer sits
inside it (/opt/skills/guides/cdna_hip_programming.md, section 5.7 item 2).
sig_hash_kernel relies on two such hand-managed facts:

* its polynomial MFMA accumulators live in AGPRs -- with VGPR accumulators
  the asm VALU blocks could be allocated onto registers an in-flight MFMA
  still reads or writes (measured wrong planes in fixed lanes, round 2);
* the `s_nop`s in pair_transpose cover the VALU-write -> DPP-read hazard of
  its v_cndmask_b32_dpp butterflies.

This module disassembles the code objects embedded in the built library
(llvm-objdump --offloading, then -d --mcpu=gfx950) and checks both facts
and, generally, every DPP read and every MFMA operand read against the VALU
writes before it, in straight-line instruction order.  Since round 6 it also
walks every function's control flow graph for registers named while a
vector-memory load into them is still in flight (vm_hazards, below: the asm
loads retired by hand-written `s_waitcnt vmcnt(N)`), and reads each kernel's
scratch and spill counts from the code object's metadata.  A compiler or
register-allocation change that breaks any of this then fails the CPU test
suite instead of corrupting CRCs or signatures silently.
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
# 2 each on gfx940/gfx950 (the `s_nop 1` pair_transpose carries).
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


# ---- in-flight vector-memory loads --------
#
# The hot kernels issue their line loads as inline asm (`global_load_dwordx4`,
# fdfs_hash.hip issue/issue_p, fdfs_md5.hip, fdfs_segcrc.hpp) and retire them
# with hand-written `s_waitcnt vmcnt(N)`.  hipcc takes an asm output register
# as written the moment the statement retires, so if register allocation ever
# copies (`v_mov`), spills (`scratch_store`) or otherwise reads or overwrites
# such a register before the wait that retires its load, that instruction sees
# the register's old contents -- silently wrong CRCs (round 5's forced
# four-wave lane kernel: DESIGN 4.1).  hipcc's own loads are covered by the
# waits it inserts itself; this check covers both alike.
#
# Model (gfx9 / CDNA: VM_CNT counts every vector-memory instruction -- loads,
# stores, atomics, LDS-DMA, flat -- and its loads return in issue order): the
# in-flight set is an ordered list, newest first; `s_waitcnt vmcnt(N)` keeps
# only the N newest.  The analysis runs forward over the function's control
# flow graph to a fixed point: at a join the lists are merged position by
# position (union of the destination registers, the longer length), which
# over-approximates what may still be in flight on any path.  Any instruction
# that names a register in flight -- as a source, a destination or a copy
# source -- is a hazard; a vector-memory instruction may name its own
# destination (two loads into one register retire in order).
VM_PREFIXES = ("global_", "buffer_", "flat_", "scratch_")
VM_MAX = 64  # the counter saturates (6 bits); issue stalls beyond it


def vm_dst(inst: str) -> set[tuple[str, int]]:
    """Registers a vector-memory instruction writes when it retires (empty for
    stores, LDS-DMA loads, cache operations and atomics without return)."""
    mnem, ops = operands(inst)
    if not ops or "store" in mnem or "_lds_" in mnem or " lds" in inst or mnem.startswith(("buffer_inv", "buffer_wb")):
        return set()
    if "_atomic" in mnem:
        return regs(ops[0]) if re.search(r"\s(sc0|glc)\b", inst) else set()
    return regs(ops[0]) if "load" in mnem else set()


def _vm_wait(inst: str) -> int | None:
    """N of an `s_waitcnt` that bounds VM_CNT, else None."""
    if not inst.startswith("s_waitcnt"):
        return None
    m = re.search(r"vmcnt\((\d+)\)", inst)
    if m:
        return int(m.group(1))
    return 0 if re.match(r"s_waitcnt\s+0\s*$", inst) else None


def _merge(a: tuple, b: tuple) -> tuple:
    if len(a) < len(b):
        a, b = b, a
    return tuple(x | b[k] if k < len(b) else x for k, x in enumerate(a))


def vm_hazards(insts: list) -> list[str]:
    """Instructions that name a register an in-flight load still writes.

    `insts` is a function body: a list of instruction strings, or of
    (text, successor-index-of-the-branch-target or None) pairs.  Branches
    (`s_branch`, `s_cbranch_*`) go to their target; conditional ones fall
    through too; `s_endpgm` / `s_setpc` end the path."""
    items = [(i, None) if isinstance(i, str) else i for i in insts]
    n = len(items)
    parsed = [operands(t) for t, _ in items]
    succ = []
    for k, ((t, tgt), (mnem, _)) in enumerate(zip(items, parsed)):
        s = []
        if mnem.startswith(("s_endpgm", "s_setpc", "s_trap")):
            pass
        elif mnem == "s_branch":
            if tgt is not None:
                s.append(tgt)
        else:
            if mnem.startswith("s_cbranch") and tgt is not None:
                s.append(tgt)
            if k + 1 < n:
                s.append(k + 1)
        succ.append(s)
    state: list = [None] * n
    if n:
        state[0] = ()
    work = [0] if n else []
    found: dict[int, str] = {}
    while work:
        k = work.pop()
        st = state[k]
        text, _ = items[k]
        mnem, ops = parsed[k]
        is_vm = mnem.startswith(VM_PREFIXES)
        live = frozenset().union(*st) if st else frozenset()
        if live:
            named = set()
            for o in ops:
                named |= regs(o)
            if is_vm:
                named -= vm_dst(text)
            if mnem.startswith(("v_movrel", "s_set_gpr_idx")):
                named = set(live)  # indexed VGPR access: any register
            bad = named & live
            if bad and k not in found:
                r = sorted(bad)[0]
                found[k] = (f"`{text}` names {r[0]}{r[1]} while a load into it is in flight "
                            f"({len(st)} vector-memory op(s) outstanding)")
        w = _vm_wait(text)
        if w is not None:
            out = st[:w]
        elif is_vm:
            out = ((frozenset(vm_dst(text)),) + st)[:VM_MAX]
        else:
            out = st
        for s in succ[k]:
            new = out if state[s] is None else _merge(state[s], out)
            if new != state[s]:
                state[s] = new
                work.append(s)
    return [found[k] for k in sorted(found)]


def disassemble_cfg(co: str) -> dict[str, list[tuple[str, int | None]]]:
    """{function symbol: [(instruction text, index of its branch target)]}:
    the body as vm_hazards takes it (branch targets from the disassembler's
    `<symbol+0xoff>` annotation, instruction addresses from its comments)."""
    out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", "--no-show-raw-insn", co], check=True,
                         capture_output=True, text=True).stdout
    funcs: dict[str, list] = {}
    cur = None
    for line in out.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            cur = m.group(2)
            funcs[cur] = (int(m.group(1), 16), [])
            continue
        if cur is None or "//" not in line:
            continue
        text, comment = line.split("//", 1)
        text = text.strip()
        ma = re.match(r"\s*([0-9A-Fa-f]+):", comment)
        if not text or text.endswith(":") or not ma:
            continue
        mt = re.search(r"<(.+)\+0x([0-9a-f]+)>", comment)
        tgt = None
        if mt and text.startswith(("s_branch", "s_cbranch")):
            tgt = funcs[cur][0] + int(mt.group(2), 16) if mt.group(1) == cur else None
        funcs[cur][1].append((int(ma.group(1), 16), text, tgt))
    res = {}
    for fn, (_, body) in funcs.items():
        index = {a: k for k, (a, _, _) in enumerate(body)}
        res[fn] = [(t, index.get(tg) if tg is not None else None) for _, t, tg in body]
    return res


def kernel_metadata(co: str) -> dict[str, dict[str, int]]:
    """{kernel symbol: {private_segment_fixed_size, vgpr_count, agpr_count,
    vgpr_spill_count, sgpr_spill_count}} from the code object's notes."""
    out = subprocess.run([os.path.join(LLVM_BIN, "llvm-readelf"), "--notes", co], check=True,
                         capture_output=True, text=True).stdout
    res: dict[str, dict[str, int]] = {}
    keys = ("private_segment_fixed_size", "vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count")
    # one kernel per `  - .key:` item of amdhsa.kernels (2-space indent);
    # its own keys sit at 4 spaces (.args items are deeper)
    for item in re.split(r"\n  - (?=\.)", out)[1:]:
        fields = dict(re.findall(r"(?:^|\n)(?:    )?\.(\w+):\s+(\S+)", item))
        if "name" in fields:
            res[fields["name"]] = {k: int(fields[k]) for k in keys if k in fields}
    return res


def check_library(lib_path: str) -> dict:
    """{"functions": n, "mfma": {kernel: [dst kinds]}, "dpp": {kernel: count},
    "setprio": {kernel: count}, "hazards": [..], "vm_hazards": [..],
    "counted_waits": {kernel: count of vmcnt(N > 0) waits}, "meta": {..}}."""
    res = {"names": [], "functions": 0, "mfma": {}, "dpp": {}, "setprio": {}, "hazards": [],
           "vm_hazards": [], "counted_waits": {}, "meta": {}}
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
            for fn, body in disassemble_cfg(co).items():
                res["vm_hazards"] += [f"{fn}: {h}" for h in vm_hazards(body)]
                nw = sum(1 for t, _ in body if (_vm_wait(t) or 0) > 0)
                if nw:
                    res["counted_waits"][fn] = res["counted_waits"].get(fn, 0) + nw
            for fn, m in kernel_metadata(co).items():
                res["meta"].setdefault(fn, m)
    return res
