// Device-side building blocks shared by the libfdfs_gpu kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "fdfs_tables.hpp"

namespace fdfs {

// Device copy of the tables: CrcTables, the complemented slice tables used by
// the segmented kernel for the signed variant (see crc_seg_kernel), and the
// matrix-core polynomial operands of sig_hash_kernel.
struct DevTables {
    CrcTables t;
    uint32_t Dc[16][256];   // Dc[p][x] = D[p][x ^ 0xFF]
    PolyMfmaTables pm;
};

// A value the code knows to be wave-uniform (a shuffle-max, say), moved to
// SGPRs so that loops and branches on it are scalar.  Left in a VGPR, a loop
// on it is exec-masked: each body is guarded by s_cbranch_execz, and a path
// that skips the body skips its asm `s_waitcnt` too (tests/isa_check.py
// vm_hazards counts such paths as loads still in flight).
__device__ __forceinline__ uint64_t uniform64(uint64_t x)
{
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
    return (uint64_t)hi << 32 | lo;
}

// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// ---- conflict-free slice-by-8: rotated, replicated byte tables ----------
// A ds_read_b32 serves lanes 0-31 and 32-63 as two groups over 32 banks
// (bank = dword address mod 32); random byte lookups into one shared table
// put ~3.5 lanes on the busiest bank (measured: 2/3 of all LDS cycles were
// conflicts).  Here lane l reads byte position (k + (l & 3)) & 3 of a data
// word at step k (a per-lane byte rotation, free inside v_perm_b32), from
// its own copy (l >> 2) & 7 of the table for that position.  Table t, copy c
// is slot t*8 + c of a 64-dword row per byte value (row e = 256 bytes), so at
// every step the 32 lanes of a group hit 32 distinct banks.
//   LDS image: dword e*64 + t*8 + c = D[8 + t][e]   (64 KiB)
//   address  = e << 8 | slot << 2  = v_perm_b32(word, off, sel): byte 1 is
//              the data byte, byte 0 the lane's slot offset.
constexpr int kRep8Dwords = 256 * 64;

// src: the 16 slice-by-16 tables (D or Dc); positions 8..15 are slice-by-8.
__device__ __forceinline__ void lds_fill_rep8(uint32_t *dst, const uint32_t *__restrict__ src)
{
    for (int i = threadIdx.x; i < kRep8Dwords; i += blockDim.x)
        dst[i] = src[(8 + ((i >> 3) & 7)) * 256 + (i >> 6)];
}

struct Rep8Lane {
    uint32_t off0, off1;  // slot byte offsets for word 0 / word 1, byte k = step k
    uint32_t sel[4];      // v_perm selectors for steps k = 0..3
};

__device__ __forceinline__ Rep8Lane rep8_lane(int lane)
{
    Rep8Lane r;
    const uint32_t b = lane & 3, c = (lane >> 2) & 7;
    r.off0 = r.off1 = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t kk = (k + b) & 3;
        r.off0 |= (((0 + kk) * 8 + c) * 4) << (8 * k);
        r.off1 |= (((4 + kk) * 8 + c) * 4) << (8 * k);
        r.sel[k] = 0x0C0C0000u | ((4u + kk) << 8) | (uint32_t)k;
    }
    return r;
}

// 8 bytes (LE words w0, w1) chained onto state c.  SAR adds the sign term.
template <bool SAR>
__device__ __forceinline__ uint32_t chain8r(const uint32_t *sR, const Rep8Lane &R, uint32_t c,
                                            uint32_t w0, uint32_t w1, uint32_t K8)
{
    const char *base = reinterpret_cast<const char *>(sR);
    const uint32_t x0 = c ^ w0;
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        v[k] = *reinterpret_cast<const uint32_t *>(base + __builtin_amdgcn_perm(x0, R.off0, R.sel[k]));
        v[4 + k] = *reinterpret_cast<const uint32_t *>(base + __builtin_amdgcn_perm(w1, R.off1, R.sel[k]));
    }
    const uint32_t s = SAR ? ((uint32_t)((int32_t)c >> 31) & K8) : 0u;
    return xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), xor3(v[6], v[7], s));
}

// 16 bytes = two slice-by-8 steps.
template <bool SAR>
__device__ __forceinline__ uint32_t chain16r(const uint32_t *sR, const Rep8Lane &R, uint32_t c,
                                             uint4 w, uint32_t K8)
{
    c = chain8r<SAR>(sR, R, c, w.x, w.y, K8);
    return chain8r<SAR>(sR, R, c, w.z, w.w, K8);
}

constexpr int kWave = 64;

__device__ __forceinline__ uint32_t shr8(uint32_t c, bool sar)
{
    return sar ? (uint32_t)((int32_t)c >> 8) : (c >> 8);
}

// One CRC32_ex byte step (storage/storage_dio.c:467) from an LDS table.
template <bool SAR>
__device__ __forceinline__ uint32_t crc_byte(const uint32_t *__restrict__ T, uint32_t c, uint32_t b)
{
    return T[(c ^ b) & 0xFFu] ^ shr8(c, SAR);
}

// 16 bytes (LE words w) chained onto state c with slice-by-16 tables D
// (LDS, [16][256]).  SAR adds the sign term the arithmetic shift leaves.
template <bool SAR>
__device__ __forceinline__ uint32_t chain16(const uint32_t *__restrict__ D, uint32_t c, uint4 w,
                                            uint32_t K16)
{
    // the XORs as v_bitop3_b32 builtins, not asm statements: hipcc schedules
    // them with the lookups and pads nothing around them
    auto xor3 = [](uint32_t a, uint32_t b, uint32_t d) { return __builtin_amdgcn_bitop3_b32(a, b, d, 0x96); };
    const uint32_t x = c ^ w.x;
    uint32_t r0 = xor3(D[0 * 256 + (x & 0xFFu)], D[1 * 256 + ((x >> 8) & 0xFFu)],
                       D[2 * 256 + ((x >> 16) & 0xFFu)]);
    uint32_t r1 = xor3(D[3 * 256 + (x >> 24)], D[4 * 256 + (w.y & 0xFFu)],
                       D[5 * 256 + ((w.y >> 8) & 0xFFu)]);
    uint32_t r2 = xor3(D[6 * 256 + ((w.y >> 16) & 0xFFu)], D[7 * 256 + (w.y >> 24)],
                       D[8 * 256 + (w.z & 0xFFu)]);
    uint32_t r3 = xor3(D[9 * 256 + ((w.z >> 8) & 0xFFu)], D[10 * 256 + ((w.z >> 16) & 0xFFu)],
                       D[11 * 256 + (w.z >> 24)]);
    r0 = xor3(r0, D[12 * 256 + (w.w & 0xFFu)], D[13 * 256 + ((w.w >> 8) & 0xFFu)]);
    r1 = xor3(r1, D[14 * 256 + ((w.w >> 16) & 0xFFu)], D[15 * 256 + (w.w >> 24)]);
    uint32_t r = xor3(r0, r1, r2) ^ r3;
    if (SAR)
        r ^= (uint32_t)((int32_t)c >> 31) & K16;
    return r;
}

// One dword of the lane fold (fdfs_tables.hpp lane_fold_exp): c'_s = x ^
// sum_{k<last} ring[(s - (32 - r_k)) & 31].  ring holds c' of the step's
// dwords 0..s-1 and of the previous step's s..31, so every source is there
// (the lag-32 one is read before slot s is overwritten).  Oldest terms first:
// the newest source is on the last bitop3 alone.  6 VALU (arithmetic shift)
// or 7 (logical) per dword, against ~7.5 VALU + 4 LDS lookups for the
// slice-by-16 fold of the same 4 bytes.
template <bool SAR>
__device__ __forceinline__ uint32_t lane_fold_dw(const uint32_t (&ring)[32], int s, uint32_t x)
{
    constexpr int nt = lane_fold_terms(SAR) - 1;  // sources
    uint32_t acc = x;
#pragma unroll
    for (int k = 0; k + 1 < nt; k += 2)
        acc = __builtin_amdgcn_bitop3_b32(acc, ring[(s - (32 - lane_fold_exp(SAR, k))) & 31],
                                          ring[(s - (32 - lane_fold_exp(SAR, k + 1))) & 31], 0x96);
    if constexpr ((nt & 1) != 0)
        acc ^= ring[(s - (32 - lane_fold_exp(SAR, nt - 1))) & 31];
    return acc;
}

// The lane's CRC state after its steps: ring = c' of its last 32 dwords
// (positions n - 32 .. n - 1).  The unfolded recursion also passed on values
// from inside that window, which the fold must not (only positions <= n - 33
// carry on), so each window dword first takes back its in-window sources
// (descending: the sources are still the unfolded c'); then the crc0 of the
// window's 128 bytes is the state.
template <bool SAR>
__device__ __forceinline__ uint32_t lane_fold_finish(const uint32_t *sD, uint32_t K16, uint32_t (&ring)[32])
{
#pragma unroll
    for (int i = 31; i >= 0; i--) {
#pragma unroll
        for (int k = 0; k < lane_fold_terms(SAR) - 1; k++) {
            const int src = i - (32 - lane_fold_exp(SAR, k));
            if (src >= 0)
                ring[i] ^= ring[src];
        }
    }
    uint32_t a = 0;
#pragma unroll
    for (int v = 0; v < 8; v++)
        a = chain16<SAR>(sD, a, make_uint4(ring[4 * v], ring[4 * v + 1], ring[4 * v + 2], ring[4 * v + 3]), K16);
    return a;
}

// Linear map given as 4 byte tables (LDS, [4][256]).
__device__ __forceinline__ uint32_t apply4(const uint32_t *__restrict__ A, uint32_t v)
{
    return (A[v & 0xFFu] ^ A[256 + ((v >> 8) & 0xFFu)]) ^
           (A[512 + ((v >> 16) & 0xFFu)] ^ A[768 + (v >> 24)]);
}

// (a << SH) + b as one full-rate v_lshl_add_u32.  Written as asm because
// hipcc otherwise folds 31*h + b / 33*h + b into v_mad_u64_u32 (a 64-bit
// multiply at a fraction of the VALU rate that also takes register pairs).
template <int SH>
__device__ __forceinline__ uint32_t lshl_add(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(SH), "v"(b));
    return r;
}

// ELFHash_ex / simple_hash_ex / Time33Hash_ex byte steps (the h[1..3] of
// CALC_HASH_CODES4, storage/storage_dio.c:475).
template <bool SAR>
__device__ __forceinline__ void h3_byte(uint32_t b, uint32_t &e, uint32_t &s, uint32_t &t)
{
    e = (e << 4) + b;
    const uint32_t x = e & 0xF0000000u;
    e ^= SAR ? (uint32_t)((int32_t)x >> 24) : (x >> 24);
    e &= ~x;
    s = lshl_add<5>(s, b) - s;  // 31*s + b
    t = lshl_add<5>(t, t) + b;  // 33*t + b
}

// ---- ELFHash_ex, byte k of word w ------------------------------------------
// t = (e << 4) + b; e = t ^ ((t >> 24) & ~0xF) (the top nibble is left
// "dirty": the next step shifts it out).  The exact step also clears the
// bits of the top nibble that were set in t, as ELFHash_ex's `h &= ~x` does;
// it is applied to the last byte of every 16-byte vector.
// One word (4 bytes) of ELF steps as a single asm block: the byte select is
// an SDWA operand of the add (v_lshl_add + v_bfe would be two half-rate
// instructions), and hipcc pads an inline-asm result with an s_nop before
// its first use, so the whole word is one statement.
#define ELF_STEP(SH, BYTE)                                                        \
    "v_lshlrev_b32 %1, 4, %0\n\t"                                                  \
    "v_add_u32_sdwa %1, %1, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" BYTE "\n\t" \
    SH " %2, 24, %1\n\t"                                                           \
    "v_bitop3_b32 %0, %2, %1, %4 bitop3:0x6c\n\t"
#define ELF_LAST(SH)                                                              \
    "v_lshlrev_b32 %1, 4, %0\n\t"                                                  \
    "v_add_u32_sdwa %1, %1, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3\n\t" \
    "v_and_b32 %0, 0xf0000000, %1\n\t"                                             \
    SH " %2, 24, %0\n\t"                                                           \
    "v_bitop3_b32 %0, %2, %0, %1 bitop3:0x12\n\t"

// bitop3:0x6c = b ^ (a & c): e = t ^ ((t >> 24) & 0xFFFFFFF0), top nibble left
// dirty (the next step shifts it out).  bitop3:0x12 = (c ^ a) & ~b: the exact
// ELFHash_ex step, x = t & 0xF0000000, e = (t ^ (x >> 24)) & ~x.
template <bool SAR, bool LAST>
__device__ __forceinline__ void elf_word4(uint32_t w, uint32_t &e)
{
    uint32_t t, y;
    const uint32_t M = 0xFFFFFFF0u;
    if constexpr (SAR && LAST)
        asm(ELF_STEP("v_ashrrev_i32", "BYTE_0") ELF_STEP("v_ashrrev_i32", "BYTE_1")
                ELF_STEP("v_ashrrev_i32", "BYTE_2") ELF_LAST("v_ashrrev_i32")
            : "+v"(e), "=&v"(t), "=&v"(y) : "v"(w), "s"(M));
    else if constexpr (SAR)
        asm(ELF_STEP("v_ashrrev_i32", "BYTE_0") ELF_STEP("v_ashrrev_i32", "BYTE_1")
                ELF_STEP("v_ashrrev_i32", "BYTE_2") ELF_STEP("v_ashrrev_i32", "BYTE_3")
            : "+v"(e), "=&v"(t), "=&v"(y) : "v"(w), "s"(M));
    else if constexpr (LAST)
        asm(ELF_STEP("v_lshrrev_b32", "BYTE_0") ELF_STEP("v_lshrrev_b32", "BYTE_1")
                ELF_STEP("v_lshrrev_b32", "BYTE_2") ELF_LAST("v_lshrrev_b32")
            : "+v"(e), "=&v"(t), "=&v"(y) : "v"(w), "s"(M));
    else
        asm(ELF_STEP("v_lshrrev_b32", "BYTE_0") ELF_STEP("v_lshrrev_b32", "BYTE_1")
                ELF_STEP("v_lshrrev_b32", "BYTE_2") ELF_STEP("v_lshrrev_b32", "BYTE_3")
            : "+v"(e), "=&v"(t), "=&v"(y) : "v"(w), "s"(M));
}
// The same four dirty-form steps, with the last byte's t >> 24 (arithmetic
// for SAR) left in y: its sign is the last t's, which is all the exact fold
// of the final state needs (elf_exact_after).
template <bool SAR>
__device__ __forceinline__ void elf_word4y(uint32_t w, uint32_t &e, uint32_t &y)
{
    uint32_t t;
    const uint32_t M = 0xFFFFFFF0u;
    if constexpr (SAR)
        asm(ELF_STEP("v_ashrrev_i32", "BYTE_0") ELF_STEP("v_ashrrev_i32", "BYTE_1")
                ELF_STEP("v_ashrrev_i32", "BYTE_2") ELF_STEP("v_ashrrev_i32", "BYTE_3")
            : "+v"(e), "=&v"(t), "=&v"(y) : "v"(w), "s"(M));
    else
        asm(ELF_STEP("v_lshrrev_b32", "BYTE_0") ELF_STEP("v_lshrrev_b32", "BYTE_1")
                ELF_STEP("v_lshrrev_b32", "BYTE_2") ELF_STEP("v_lshrrev_b32", "BYTE_3")
            : "+v"(e), "=&v"(t), "=&v"(y) : "v"(w), "s"(M));
}
#undef ELF_STEP
#undef ELF_LAST

// A whole 16-byte vector of dirty-form steps in one asm statement (hipcc
// pads the boundary between two asm statements with an s_nop: one boundary
// per vector instead of four); y as in elf_word4y.
#define ELF_WORD(SH, W) \
    ELF_STEP_W(SH, "BYTE_0", W) ELF_STEP_W(SH, "BYTE_1", W) ELF_STEP_W(SH, "BYTE_2", W) ELF_STEP_W(SH, "BYTE_3", W)
#define ELF_STEP_W(SH, BYTE, W)                                                   \
    "v_lshlrev_b32 %1, 4, %0\n\t"                                                  \
    "v_add_u32_sdwa %1, %1, %" W " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" BYTE "\n\t" \
    SH " %2, 24, %1\n\t"                                                           \
    "v_bitop3_b32 %0, %2, %1, %7 bitop3:0x6c\n\t"
template <bool SAR>
__device__ __forceinline__ void elf_vec16y(uint4 q, uint32_t &e, uint32_t &y)
{
    uint32_t t;
    const uint32_t M = 0xFFFFFFF0u;
    if constexpr (SAR)
        asm(ELF_WORD("v_ashrrev_i32", "3") ELF_WORD("v_ashrrev_i32", "4") ELF_WORD("v_ashrrev_i32", "5")
                ELF_WORD("v_ashrrev_i32", "6")
            : "+v"(e), "=&v"(t), "=&v"(y) : "v"(q.x), "v"(q.y), "v"(q.z), "v"(q.w), "s"(M));
    else
        asm(ELF_WORD("v_lshrrev_b32", "3") ELF_WORD("v_lshrrev_b32", "4") ELF_WORD("v_lshrrev_b32", "5")
                ELF_WORD("v_lshrrev_b32", "6")
            : "+v"(e), "=&v"(t), "=&v"(y) : "v"(q.x), "v"(q.y), "v"(q.z), "v"(q.w), "s"(M));
}
#undef ELF_WORD
#undef ELF_STEP_W

// The exact ELFHash_ex state from a dirty-form one.  The two differ in bits
// 28-31 only.  The exact step leaves them ~t's top nibble when the last t was
// negative (SAR: x >> 24 sign-extends into them) -- as the dirty form does --
// and clear otherwise.  y = the last step's t >> 24, or any negative value
// when the state is already exact.
__device__ __forceinline__ uint32_t elf_exact_after(uint32_t e, uint32_t y)
{
    return (int32_t)y < 0 ? e : (e & 0x0FFFFFFFu);
}

// The same word of ELF steps in plain C, for waves bound by ELF's dependent
// chain rather than by issue: hipcc emits v_lshl_add_u32 (shift + byte add in
// one op), v_ashrrev / v_lshrrev and v_bitop3 -- three ops on the chain per
// byte instead of four -- and extracts the bytes (v_and / v_bfe / v_lshr)
// off the chain, where they fill its latency gaps.
template <bool SAR, bool LAST>
__device__ __forceinline__ void elf_word4_chain(uint32_t w, uint32_t &e)
{
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t t = (e << 4) + ((w >> (8 * k)) & 0xFFu);
        if (LAST && k == 3) {
            const uint32_t x = t & 0xF0000000u;
            e = (t ^ (SAR ? (uint32_t)((int32_t)x >> 24) : (x >> 24))) & ~x;
        } else {
            e = t ^ ((SAR ? (uint32_t)((int32_t)t >> 24) : (t >> 24)) & 0xFFFFFFF0u);
        }
    }
}

// elf_word4_chain<SAR, false> that also leaves the last byte's t >> 24 in y.
template <bool SAR>
__device__ __forceinline__ void elf_word4_chain_y(uint32_t w, uint32_t &e, uint32_t &y)
{
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t t = (e << 4) + ((w >> (8 * k)) & 0xFFu);
        const uint32_t yt = SAR ? (uint32_t)((int32_t)t >> 24) : (t >> 24);
        e = t ^ (yt & 0xFFFFFFF0u);
        if (k == 3)
            y = yt;
    }
}

// ---- simple_hash_ex (M = 31) / Time33Hash_ex (M = 33), one word -----------
// h4 = M^4 h + M^3 b0 + M^2 b1 + M b2 + b3 (mod 2^32).  M^3 < 2^16, so the
// word polynomial is two v_dot4 byte planes.
template <uint32_t M>
struct Poly4 {
    static constexpr uint32_t c3 = M * M * M, c2 = M * M, c1 = M;
    static constexpr uint32_t lo = (c3 & 0xFFu) | ((c2 & 0xFFu) << 8) | ((c1 & 0xFFu) << 16) | (1u << 24);
    static constexpr uint32_t hi = ((c3 >> 8) & 0xFFu) | (((c2 >> 8) & 0xFFu) << 8);
    static constexpr uint32_t m4 = M * M * M * M;
    static_assert(c3 < 65536 && c1 < 256, "two planes");
};

template <uint32_t M>
__device__ __forceinline__ uint32_t poly_word(uint32_t h, uint32_t w)
{
    const uint32_t hi = __builtin_amdgcn_udot4(w, Poly4<M>::hi, 0u, false);
    return __builtin_amdgcn_udot4(w, Poly4<M>::lo, h * Poly4<M>::m4 + (hi << 8), false);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// m^e mod 2^32 (simple_hash / Time33 multipliers raised to a length).
__device__ __forceinline__ uint32_t pow_dev(uint32_t m, uint64_t e)
{
    uint32_t r = 1;
    for (; e; e >>= 1, m *= m)
        if (e & 1)
            r *= m;
    return r;
}

// One thread's GF(2) advance of a CRC32_ex state by `nbytes` zero bytes,
// v -> M^nbytes v, from the matrix powers M^(2^k) (columns in t.MPOW).  Used
// where a chunk's state must be carried over the chunk: CRC32_ex(d, X) =
// M^|d| X ^ CRC32_ex(d, 0) for both shift variants (linear over GF(2)).
__device__ __forceinline__ uint32_t advance_bytes(const CrcTables &t, uint32_t v, uint64_t nbytes)
{
    for (int k = 0; nbytes && k < 48; k++, nbytes >>= 1) {
        if (!(nbytes & 1))
            continue;
        uint32_t r = 0;
#pragma unroll 8
        for (int c = 0; c < 32; c++)
            r ^= (0u - ((v >> c) & 1u)) & t.MPOW[k][c];
        v = r;
    }
    return v;
}

// fdfs_gpu_file_state.md5_count += 8 * nbytes (two u32 words, low first).
__device__ __forceinline__ void count_add(uint32_t (&cnt)[2], uint64_t nbytes)
{
    const uint64_t c = ((uint64_t)cnt[1] << 32 | cnt[0]) + (nbytes << 3);
    cnt[0] = (uint32_t)c;
    cnt[1] = (uint32_t)(c >> 32);
}

// Pair transpose of one quarter line (sig_hash_kernel, crc_lane_kernel): lane
// j of a lane pair holds in r0 / r1 piece j of pair-file 0 / 1; afterwards
// lane j holds pieces 0 and 1 of its own file, in r0 and t.  One stage (lane
// xor 1): 8 VALU per two vectors (round 4: the quad form's two stages took 16).
__device__ __forceinline__ void pair_transpose(uint32_t (&r0)[4], const uint32_t (&r1)[4], uint32_t (&t)[4])
{
#define PD(D, S0, S1) "v_cndmask_b32_dpp %[" D "], %[" S0 "], %[" S1 "], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
    asm volatile(
        "s_nop 1\n\t"
        "s_mov_b32 vcc_lo, 0xaaaaaaaa\n\ts_mov_b32 vcc_hi, 0xaaaaaaaa\n\t"  // odd lanes keep r1
        PD("t0", "a0", "b0") PD("t1", "a1", "b1") PD("t2", "a2", "b2") PD("t3", "a3", "b3")
        "s_mov_b32 vcc_lo, 0x55555555\n\ts_mov_b32 vcc_hi, 0x55555555\n\t"  // even lanes keep r0
        PD("a0", "b0", "a0") PD("a1", "b1", "a1") PD("a2", "b2", "a2") PD("a3", "b3", "a3")
        : [a0] "+v"(r0[0]), [a1] "+v"(r0[1]), [a2] "+v"(r0[2]), [a3] "+v"(r0[3]),
          [t0] "=&v"(t[0]), [t1] "=&v"(t[1]), [t2] "=&v"(t[2]), [t3] "=&v"(t[3])
        : [b0] "v"(r1[0]), [b1] "v"(r1[1]), [b2] "v"(r1[2]), [b3] "v"(r1[3])
        : "vcc");
#undef PD
}

// Cooperative global -> LDS copy of `ndw` dwords.
__device__ __forceinline__ void lds_fill(uint32_t *dst, const uint32_t *__restrict__ src, int ndw)
{
    for (int i = threadIdx.x; i < ndw; i += blockDim.x)
        dst[i] = src[i];
}

}  // namespace fdfs
