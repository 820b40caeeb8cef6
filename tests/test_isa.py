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
    assert len(hash_kernels) >= 6  # {signed, unsigned} x {one-shot, quad loads, state}
    for k, kinds in hash_kernels.items():
        assert kinds and set(kinds) == {"a"}, k


def test_no_valu_to_dpp_or_mfma_hazard(isa):
    """No DPP read (quad_transpose's v_cndmask_b32_dpp butterflies, the
    compiler's own DPP moves) and no MFMA operand read follows the VALU write
    of its register by fewer than the required wait states."""
    assert sum(v for k, v in isa["dpp"].items() if "sig_hash_kernel" in k) > 100
    assert isa["hazards"] == []


def test_shipped_kernels_carry_no_probe_code(isa):
    """the probe knobs are compiled into the probe build only.
    The production md5_pair_kernel is the PM 0 instantiation alone (PM is a
    template parameter).  Round 4 made its longest-remaining-first issue
    priority production (prio_by_remaining): md5_pair_kernel is
    the only shipped kernel that changes its priority."""
    pair = [k for k in isa["names"] if "md5_pair_kernel" in k]
    assert pair, "md5_pair_kernel not found in the shipped code object"
    assert all(("Lb1ELi0E" in k or "Lb0ELi0E" in k) for k in pair), pair
    assert isa["setprio"], "the pair kernel's priority policy is missing"
    assert all("md5_pair_kernel" in k for k in isa["setprio"]), isa["setprio"]
    # round 4's measured-and-not-kept variants live in the probe build only
    for probe in ("sig_split_kernel", "tail_plan_kernel", "dp_tile_kernelILb0E", "dp_split_kernelILi1024ELb1E"):
        assert not any(probe in k for k in isa["names"]), probe


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
