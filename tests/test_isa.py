"""CPU: the inline-asm hazards of the hash kernel, checked on the gfx950
code objects the library ships (tests/isa_check.py)."""
import pytest

from fastdfs_amd import _lib

import isa_check as I


@pytest.fixture(scope="module")
def isa():
    return I.check_library(_lib.LIB_PATH)


def test_hash_kernel_accumulators_are_agprs(isa):
    """Every sig_hash_kernel instantiation keeps its polynomial MFMA
    accumulators in AGPRs (a "v"-constrained asm operand cannot be one, so
    the asm VALU blocks can never land on a register an in-flight MFMA
    uses)."""
    hash_kernels = {k: v for k, v in isa["mfma"].items() if "sig_hash_kernel" in k}
    assert len(hash_kernels) >= 4  # {signed, unsigned} x {one-shot, state}
    for k, kinds in hash_kernels.items():
        assert kinds and set(kinds) == {"a"}, k


def test_no_valu_to_dpp_or_mfma_hazard(isa):
    """No DPP read (pair_transpose's v_cndmask_b32_dpp butterflies, the
    compiler's own DPP moves) and no MFMA operand read follows the VALU write
    of its register by fewer than the required wait states."""
    assert sum(v for k, v in isa["dpp"].items() if "sig_hash_kernel" in k) > 100
    assert isa["hazards"] == []


def test_shipped_kernels_carry_no_probe_code(isa):
    """the product sources hold only the forms that
    ship; measured variants are patches applied by `make probes`
    (fastdfs_amd/csrc/probes/*.patch).  Each production kernel template is
    instantiated only on what ships (shift variant, state mode, NB bins, GM
    gidx mode): no probe-mode parameter is left in a shipped name.  Round 4
    made md5_pair_kernel's longest-remaining-first issue priority production
    (prio_by_remaining); round 6's chain workgroups (md5_chain_wg
    in md5_pair_kernel and md5_stage_kernel, elf_chain_wg in sig_hash_kernel) raise
    their chain wave's: those are the only shipped kernels that change
    their priority."""
    names = isa["names"]
    pair = [k for k in names if "md5_pair_kernel" in k]
    assert pair, "md5_pair_kernel not found in the shipped code object"
    assert all(k.startswith(("_ZN4fdfs15md5_pair_kernelILb1EEEv", "_ZN4fdfs15md5_pair_kernelILb0EEEv")) for k in pair), pair
    assert all(("ILb0ELb" in k or "ILb1ELb" in k) and "ELi" not in k for k in names if "sig_hash_kernel" in k)
    assert all(k.startswith(("_ZN4fdfs14crc_seg_kernelILb1EEEv", "_ZN4fdfs14crc_seg_kernelILb0EEEv"))
               for k in names if "crc_seg_kernel" in k)
    assert isa["setprio"], "the pair kernel's priority policy is missing"
    assert any("md5_pair_kernel" in k for k in isa["setprio"]), isa["setprio"]
    assert all(any(m in k for m in ("md5_pair_kernel", "md5_stage_kernel", "sig_hash_kernel"))
               for k in isa["setprio"]), isa["setprio"]
    # measured-and-not-kept variants of rounds 1-4 are gone from the product
    for probe in ("sig_split_kernel", "tail_plan_kernel", "dp_tile_kernelILb", "dp_split_kernelILi1024ELb"):
        assert not any(probe in k for k in names), probe


DPP = "v_cndmask_b32_dpp v6, v5, v7, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
MFMA = "v_mfma_i32_16x16x64_i8 a[0:3], v[60:63], v[110:113], a[0:3]"


@pytest.mark.parametrize("seq,nbad", [
    (["v_add_u32_e32 v5, v1, v2", DPP], 1),
    (["v_add_u32_e32 v5, v1, v2", "s_mov_b32 vcc_lo, 0x55555555", DPP], 1),
    (["v_add_u32_e32 v5, v1, v2", "s_nop 1", DPP], 0),
    (["v_add_u32_e32 v5, v1, v2", "s_mov_b32 vcc_lo, 1", "s_mov_b32 vcc_hi, 1", DPP], 0),
    (["v_add_u32_e32 v7, v1, v2", DPP], 0),  # src1 is read normally
    (["v_bitop3_b32 v61, v1, v2, s4 bitop3:0x6a", MFMA], 1),
    (["v_bitop3_b32 v112, v1, v2, s4 bitop3:0x6a", "s_nop 0", MFMA], 1),
    (["v_bitop3_b32 v61, v1, v2, s4 bitop3:0x6a", "s_nop 1", MFMA], 0),
    (["v_add_u32_e32 v5, v1, v2", "s_cbranch_scc1 0", DPP], 0),  # straight-line order only
])
def test_checker_finds_planted_hazards(seq, nbad):
    assert len(I.hazards(seq)) == nbad


# ---- loads still in flight ----------

HOT = ("crc_lane_kernel", "sig_hash_kernel", "md5_pair_kernel", "md5_stage_kernel", "crc_seg_kernel",
       "crc_tab_kernel")


def test_no_register_named_while_its_load_is_in_flight(isa):
    """The hot kernels' line loads are inline asm retired by hand-written
    `s_waitcnt vmcnt(N)`; hipcc takes their registers as written when the
    asm statement retires.  No instruction of any shipped kernel -- a copy, a
    spill, a DPP transpose, an overwrite -- names a register before the
    wait that retires the load into it, on any path of the control flow
    graph (isa_check.vm_hazards).  The round-5 forced-four-wave lane kernel
    failed exactly this (profiles/r06/isa_w4_variant.txt)."""
    for k in ("crc_lane_kernel", "sig_hash_kernel", "md5_pair_kernel", "crc_seg_kernel"):
        waits = [v for fn, v in isa["counted_waits"].items() if k in fn]
        assert waits and min(waits) >= 8, (k, waits)  # the checker sees the counted waits
    assert isa["vm_hazards"] == []


def test_hot_kernels_use_no_scratch(isa):
    """No spill in the kernels whose asm loads stay in flight across other
    code: a spill of such a register stores its old contents."""
    hot = {fn: m for fn, m in isa["meta"].items() if any(h in fn for h in HOT)}
    assert len(hot) >= 16, sorted(hot)
    for fn, m in hot.items():
        assert m["private_segment_fixed_size"] == 0 and m["vgpr_spill_count"] == 0, (fn, m)


LD = "global_load_dwordx4 v[44:47], v[2:3], off"
LD2 = "global_load_dwordx4 v[48:51], v[2:3], off offset:16"


@pytest.mark.parametrize("seq,nbad", [
    ([LD, "v_xor_b32_e32 v1, v44, v2"], 1),                                  # read before the wait
    ([LD, "s_waitcnt vmcnt(0)", "v_xor_b32_e32 v1, v44, v2"], 0),
    ([LD, LD2, "s_waitcnt vmcnt(1)", "v_xor_b32_e32 v1, v44, v2"], 0),       # the older load retired
    ([LD, LD2, "s_waitcnt vmcnt(1)", "v_xor_b32_e32 v1, v48, v2"], 1),       # the newer one is not
    ([LD, "global_store_dword v[4:5], v6, off", "s_waitcnt vmcnt(1)", "v_mov_b32_e32 v1, v45"], 0),  # stores count
    ([LD, "scratch_store_dwordx4 off, v[44:47], off", "s_waitcnt vmcnt(0)"], 1),  # round 5's w4 spill
    ([LD, "v_mov_b32_e32 v60, v46", "s_waitcnt vmcnt(0)"], 1),                # a copy of it
    ([LD, "v_mov_b32_e32 v46, v60", "s_waitcnt vmcnt(0)"], 1),                # an overwrite of it
    ([LD, "v_cndmask_b32_dpp v41, v45, v51, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"], 1),
    ([LD, "global_load_dwordx4 v[44:47], v[8:9], off", "s_waitcnt vmcnt(0)"], 0),  # loads retire in order
    ([LD, "global_load_lds_dwordx4 v[8:9], off", "s_waitcnt vmcnt(1)", "v_mov_b32_e32 v1, v44"], 0),
    ([LD, "s_waitcnt lgkmcnt(0)", "v_mov_b32_e32 v1, v44"], 1),              # the wrong counter
    (["global_atomic_add v7, v[2:3], v4, off sc0", "v_mov_b32_e32 v1, v7"], 1),  # atomic with return
    (["global_atomic_add v[2:3], v7, off", "v_mov_b32_e32 v7, 0"], 0),        # without: v7 is data
    # control flow: (text, branch target index)
    ([(LD, None), ("s_cbranch_execz 1", 3), ("s_waitcnt vmcnt(0)", None), ("v_mov_b32_e32 v1, v44", None)], 1),
    ([(LD, None), ("s_cbranch_scc1 1", 3), ("s_waitcnt vmcnt(0)", None), ("s_waitcnt vmcnt(0)", None),
      ("v_mov_b32_e32 v1, v44", None)], 0),
    # a loop whose loads are consumed after the back edge: waited / not waited
    ([("s_waitcnt vmcnt(0)", None), ("v_mov_b32_e32 v1, v44", None), (LD, None), ("s_cbranch_scc1 0", 0),
      ("s_waitcnt vmcnt(0)", None), ("s_endpgm", None)], 0),
    ([("v_mov_b32_e32 v1, v44", None), (LD, None), ("s_cbranch_scc1 0", 0), ("s_waitcnt vmcnt(0)", None),
      ("s_endpgm", None)], 1),
])
def test_checker_finds_planted_inflight_reads(seq, nbad):
    assert len(I.vm_hazards(seq)) == nbad
