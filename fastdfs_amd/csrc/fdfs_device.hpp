// Device-side building blocks shared by the libfdfs_gpu kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "fdfs_tables.hpp"

namespace fdfs {

// Device copy of the tables: CrcTables plus the complemented slice tables
// used by the segmented kernel for the signed variant (see crc_seg_kernel).
struct DevTables {
    CrcTables t;
    uint32_t Dc[16][256];   // Dc[p][x] = D[p][x ^ 0xFF]
    // nibble form of D / Dc: N[2p+h][x] = D[p][x << 4h]; replicated 32x per
    // lane bank in LDS by the kernels (conflict-free lookups)
    uint32_t N[32][16];
    uint32_t Nc[32][16];
};

constexpr int kNibTables = 32;
constexpr int kNibDwords = kNibTables * 16 * 32;  // 64 KiB of LDS

// Fill the lane-bank-replicated nibble tables: dword t*512 + x*32 + r = src[t][x].
__device__ __forceinline__ void lds_fill_nib(uint32_t *dst, const uint32_t *__restrict__ src)
{
    for (int i = threadIdx.x; i < kNibDwords; i += blockDim.x)
        dst[i] = src[(i >> 9) * 16 + ((i >> 5) & 15)];
}

// chain16 through the replicated nibble tables: lane l reads only bank l%32.
// lb = (lane & 31) * 4.  32 lookups per 16 bytes, no bank conflicts.
template <bool SAR>
__device__ __forceinline__ uint32_t chain16n(const uint32_t *sN, uint32_t lb, uint32_t c, uint4 w,
                                             uint32_t K16)
{
    const char *base = reinterpret_cast<const char *>(sN);
    const uint32_t x = c ^ w.x;
    const uint32_t words[4] = {x, w.y, w.z, w.w};
    uint32_t r[4] = {0, 0, 0, 0};
#pragma unroll
    for (int wi = 0; wi < 4; wi++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t a = (((words[wi] >> (4 * k)) & 0xFu) << 7) | lb;
            r[k & 3] ^= *reinterpret_cast<const uint32_t *>(base + a + (wi * 8 + k) * 2048);
        }
    }
    uint32_t v = (r[0] ^ r[1]) ^ (r[2] ^ r[3]);
    if (SAR)
        v ^= (uint32_t)((int32_t)c >> 31) & K16;
    return v;
}

// ---- nibble tables addressed with one v_perm_b32 per lookup ------------
// Layout (64 KiB): table pair q = t/2 occupies 4 KiB; entry x of table t,
// replica r (= lane % 32) sits at byte q*4096 + x*256 + (t&1)*128 + r*4.
// Every lane reads only its own bank, and the address lb + (nibble << 8) is a
// single byte permute of {nibble byte, lb byte}: v_perm_b32(v, lb, sel).
constexpr int kNibPDwords = 16 * 1024;

__device__ __forceinline__ void lds_fill_nibp(uint32_t *dst, const uint32_t *__restrict__ src)
{
    for (int i = threadIdx.x; i < kNibPDwords; i += blockDim.x) {
        const int q = i >> 10, x = (i >> 6) & 15, h = (i >> 5) & 1;
        dst[i] = src[(2 * q + h) * 16 + x];
    }
}

// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

template <bool SAR>
__device__ __forceinline__ uint32_t chain16p(const uint32_t *sN, uint32_t lb, uint32_t c, uint4 w,
                                             uint32_t K16)
{
    const char *base = reinterpret_cast<const char *>(sN);
    const uint32_t words[4] = {c ^ w.x, w.y, w.z, w.w};
    uint32_t r0 = 0, r1 = 0;
#pragma unroll
    for (int wi = 0; wi < 4; wi++) {
        const uint32_t lo = words[wi] & 0x0F0F0F0Fu;
        const uint32_t hi = (words[wi] >> 4) & 0x0F0F0F0Fu;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int p = 4 * wi + j;  // byte position in the 16-byte chunk
            const uint32_t sel = 0x0C0C0000u | ((4u + j) << 8);
            const uint32_t alo = __builtin_amdgcn_perm(lo, lb, sel);
            const uint32_t ahi = __builtin_amdgcn_perm(hi, lb, sel);
            const uint32_t vlo = *reinterpret_cast<const uint32_t *>(base + alo + p * 4096);
            const uint32_t vhi = *reinterpret_cast<const uint32_t *>(base + ahi + p * 4096 + 128);
            if (j & 1)
                r1 = xor3(r1, vlo, vhi);
            else
                r0 = xor3(r0, vlo, vhi);
        }
    }
    uint32_t v = r0 ^ r1;
    if (SAR)
        v ^= (uint32_t)((int32_t)c >> 31) & K16;
    return v;
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

template <bool SAR>
__device__ __forceinline__ void h3_word(uint32_t w, uint32_t &e, uint32_t &s, uint32_t &t)
{
    h3_byte<SAR>(w & 0xFFu, e, s, t);
    h3_byte<SAR>((w >> 8) & 0xFFu, e, s, t);
    h3_byte<SAR>((w >> 16) & 0xFFu, e, s, t);
    h3_byte<SAR>(w >> 24, e, s, t);
}

// ---- simple_hash / Time33 over 16 bytes at once ------------------------
// Both are linear recurrences h = m*h + b over Z/2^32 (m = 31 / 33), so
//   h_16 = m^16 * h_0 + sum_p m^(15-p) * b_p   (mod 2^32).
// Each coefficient is split into byte planes; plane j of the sum is
// sum_p byte_j(m^(15-p)) * b_p, four bytes at a time with v_dot4_u32_u8.
// Planes whose coefficients are all zero are folded away at compile time.
constexpr uint32_t pow_mod32(uint32_t m, int e)
{
    uint32_t r = 1;
    for (int i = 0; i < e; i++)
        r *= m;
    return r;
}

template <uint32_t M>
struct Poly16 {
    // packed[w][j] = bytes k=0..3 of plane j of the coefficients of word w
    static constexpr uint32_t coef(int w, int j)
    {
        uint32_t r = 0;
        for (int k = 0; k < 4; k++)
            r |= ((pow_mod32(M, 15 - (4 * w + k)) >> (8 * j)) & 0xFFu) << (8 * k);
        return r;
    }
    static constexpr uint32_t m16 = pow_mod32(M, 16);
};

template <uint32_t M>
__device__ __forceinline__ uint32_t poly16_step(uint32_t h, uint4 q)
{
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
    uint32_t a[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (Poly16<M>::coef(i, j) != 0)
                a[j] = __builtin_amdgcn_udot4(w[i], Poly16<M>::coef(i, j), a[j], false);
    const uint32_t sum = a[0] + (a[1] << 8) + (a[2] << 16) + (a[3] << 24);
    return h * Poly16<M>::m16 + sum;
}

// ELFHash_ex alone (the one hash of CALC_HASH_CODES4 with no parallel form).
template <bool SAR>
__device__ __forceinline__ void elf_byte(uint32_t b, uint32_t &e)
{
    e = (e << 4) + b;
    const uint32_t x = e & 0xF0000000u;
    e ^= SAR ? (uint32_t)((int32_t)x >> 24) : (x >> 24);
    e &= ~x;
}

template <bool SAR>
__device__ __forceinline__ void elf_word(uint32_t w, uint32_t &e)
{
    elf_byte<SAR>(w & 0xFFu, e);
    elf_byte<SAR>((w >> 8) & 0xFFu, e);
    elf_byte<SAR>((w >> 16) & 0xFFu, e);
    elf_byte<SAR>(w >> 24, e);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// Cooperative global -> LDS copy of `ndw` dwords.
__device__ __forceinline__ void lds_fill(uint32_t *dst, const uint32_t *__restrict__ src, int ndw)
{
    for (int i = threadIdx.x; i < ndw; i += blockDim.x)
        dst[i] = src[i];
}

}  // namespace fdfs
