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
    """No DPP read (quad_transpose's v_cndmask_b32_dpp butterflies, the
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
    (prio_by_remaining): it is the only shipped kernel that
    changes its priority."""
    names = isa["names"]
    pair = [k for k in names if "md5_pair_kernel" in k]
    assert pair, "md5_pair_kernel not found in the shipped code object"
    assert all(k.startswith(("_ZN4fdfs15md5_pair_kernelILb1EEEv", "_ZN4fdfs15md5_pair_kernelILb0EEEv")) for k in pair), pair
    assert all(("ILb0ELb" in k or "ILb1ELb" in k) and "ELi" not in k for k in names if "sig_hash_kernel" in k)
    assert all(k.startswith(("_ZN4fdfs14crc_seg_kernelILb1EEEv", "_ZN4fdfs14crc_seg_kernelILb0EEEv"))
               for k in names if "crc_seg_kernel" in k)
    assert isa["setprio"], "the pair kernel's priority policy is missing"
    assert all("md5_pair_kernel" in k for k in isa["setprio"]), isa["setprio"]
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
