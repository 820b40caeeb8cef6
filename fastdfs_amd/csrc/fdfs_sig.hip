// libfdfs_gpu signature kernels (gfx950).
//
//  * sig_lane_kernel<SAR, METHOD>: one LANE per file (files size-sorted so a
//    wave's 64 files have near-equal length).  Computes CRC32 + the 4-way
//    hash codes (METHOD 1) or CRC32 + MD5 (METHOD 2) in one pass over the
//    file and writes crc, the 24-byte signature and the raw codes.  ELFHash
//    and MD5 are sequential per file, so a lane per file is the only
//    decomposition that keeps them exact.
//  * crc_seg_kernel<SAR>: CRC32 only (the default upload path), one WAVE per
//    64 KiB segment of a file, coalesced 4 KiB strides, slice-by-16 tables in
//    LDS, a 6-level GF(2) combine across the wave, and a GF(2) matrix-power
//    advance to combine segments of large files.
//  * planning kernels: size-bin counting sort (lane path), per-file segment
//    counts + exclusive scan (segment path).
//
// Reference call sites replaced: storage/storage_dio.c:465-515 (CRC32_ex,
// CALC_HASH_CODES4, my_md5_update, *_FINAL) and
// storage/storage_service.c:106-120 (STORAGE_GEN_FILE_SIGNATURE).
#include "fdfs_device.hpp"
#include "fdfs_kernels.hpp"

#include <cstdlib>

namespace fdfs {

// ----------------------------------------------------------------- MD5 core

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s)
{
    return __builtin_amdgcn_alignbit(x, x, 32 - s);
}

#define MD5_F(b, c, d) ((d) ^ ((b) & ((c) ^ (d))))
#define MD5_G(b, c, d) ((c) ^ ((d) & ((b) ^ (c))))
#define MD5_H(b, c, d) ((b) ^ (c) ^ (d))
#define MD5_I(b, c, d) ((c) ^ ((b) | ~(d)))
#define MD5_STEP(FN, a, b, c, d, m, k, s) a = (b) + rotl((a) + FN(b, c, d) + (m) + (k), s)

__device__ __forceinline__ void md5_compress(uint32_t st[4], const uint32_t m[16])
{
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    MD5_STEP(MD5_F, a, b, c, d, m[0], 0xd76aa478u, 7);
    MD5_STEP(MD5_F, d, a, b, c, m[1], 0xe8c7b756u, 12);
    MD5_STEP(MD5_F, c, d, a, b, m[2], 0x242070dbu, 17);
    MD5_STEP(MD5_F, b, c, d, a, m[3], 0xc1bdceeeu, 22);
    MD5_STEP(MD5_F, a, b, c, d, m[4], 0xf57c0fafu, 7);
    MD5_STEP(MD5_F, d, a, b, c, m[5], 0x4787c62au, 12);
    MD5_STEP(MD5_F, c, d, a, b, m[6], 0xa8304613u, 17);
    MD5_STEP(MD5_F, b, c, d, a, m[7], 0xfd469501u, 22);
    MD5_STEP(MD5_F, a, b, c, d, m[8], 0x698098d8u, 7);
    MD5_STEP(MD5_F, d, a, b, c, m[9], 0x8b44f7afu, 12);
    MD5_STEP(MD5_F, c, d, a, b, m[10], 0xffff5bb1u, 17);
    MD5_STEP(MD5_F, b, c, d, a, m[11], 0x895cd7beu, 22);
    MD5_STEP(MD5_F, a, b, c, d, m[12], 0x6b901122u, 7);
    MD5_STEP(MD5_F, d, a, b, c, m[13], 0xfd987193u, 12);
    MD5_STEP(MD5_F, c, d, a, b, m[14], 0xa679438eu, 17);
    MD5_STEP(MD5_F, b, c, d, a, m[15], 0x49b40821u, 22);

    MD5_STEP(MD5_G, a, b, c, d, m[1], 0xf61e2562u, 5);
    MD5_STEP(MD5_G, d, a, b, c, m[6], 0xc040b340u, 9);
    MD5_STEP(MD5_G, c, d, a, b, m[11], 0x265e5a51u, 14);
    MD5_STEP(MD5_G, b, c, d, a, m[0], 0xe9b6c7aau, 20);
    MD5_STEP(MD5_G, a, b, c, d, m[5], 0xd62f105du, 5);
    MD5_STEP(MD5_G, d, a, b, c, m[10], 0x02441453u, 9);
    MD5_STEP(MD5_G, c, d, a, b, m[15], 0xd8a1e681u, 14);
    MD5_STEP(MD5_G, b, c, d, a, m[4], 0xe7d3fbc8u, 20);
    MD5_STEP(MD5_G, a, b, c, d, m[9], 0x21e1cde6u, 5);
    MD5_STEP(MD5_G, d, a, b, c, m[14], 0xc33707d6u, 9);
    MD5_STEP(MD5_G, c, d, a, b, m[3], 0xf4d50d87u, 14);
    MD5_STEP(MD5_G, b, c, d, a, m[8], 0x455a14edu, 20);
    MD5_STEP(MD5_G, a, b, c, d, m[13], 0xa9e3e905u, 5);
    MD5_STEP(MD5_G, d, a, b, c, m[2], 0xfcefa3f8u, 9);
    MD5_STEP(MD5_G, c, d, a, b, m[7], 0x676f02d9u, 14);
    MD5_STEP(MD5_G, b, c, d, a, m[12], 0x8d2a4c8au, 20);

    MD5_STEP(MD5_H, a, b, c, d, m[5], 0xfffa3942u, 4);
    MD5_STEP(MD5_H, d, a, b, c, m[8], 0x8771f681u, 11);
    MD5_STEP(MD5_H, c, d, a, b, m[11], 0x6d9d6122u, 16);
    MD5_STEP(MD5_H, b, c, d, a, m[14], 0xfde5380cu, 23);
    MD5_STEP(MD5_H, a, b, c, d, m[1], 0xa4beea44u, 4);
    MD5_STEP(MD5_H, d, a, b, c, m[4], 0x4bdecfa9u, 11);
    MD5_STEP(MD5_H, c, d, a, b, m[7], 0xf6bb4b60u, 16);
    MD5_STEP(MD5_H, b, c, d, a, m[10], 0xbebfbc70u, 23);
    MD5_STEP(MD5_H, a, b, c, d, m[13], 0x289b7ec6u, 4);
    MD5_STEP(MD5_H, d, a, b, c, m[0], 0xeaa127fau, 11);
    MD5_STEP(MD5_H, c, d, a, b, m[3], 0xd4ef3085u, 16);
    MD5_STEP(MD5_H, b, c, d, a, m[6], 0x04881d05u, 23);
    MD5_STEP(MD5_H, a, b, c, d, m[9], 0xd9d4d039u, 4);
    MD5_STEP(MD5_H, d, a, b, c, m[12], 0xe6db99e5u, 11);
    MD5_STEP(MD5_H, c, d, a, b, m[15], 0x1fa27cf8u, 16);
    MD5_STEP(MD5_H, b, c, d, a, m[2], 0xc4ac5665u, 23);

    MD5_STEP(MD5_I, a, b, c, d, m[0], 0xf4292244u, 6);
    MD5_STEP(MD5_I, d, a, b, c, m[7], 0x432aff97u, 10);
    MD5_STEP(MD5_I, c, d, a, b, m[14], 0xab9423a7u, 15);
    MD5_STEP(MD5_I, b, c, d, a, m[5], 0xfc93a039u, 21);
    MD5_STEP(MD5_I, a, b, c, d, m[12], 0x655b59c3u, 6);
    MD5_STEP(MD5_I, d, a, b, c, m[3], 0x8f0ccc92u, 10);
    MD5_STEP(MD5_I, c, d, a, b, m[10], 0xffeff47du, 15);
    MD5_STEP(MD5_I, b, c, d, a, m[1], 0x85845dd1u, 21);
    MD5_STEP(MD5_I, a, b, c, d, m[8], 0x6fa87e4fu, 6);
    MD5_STEP(MD5_I, d, a, b, c, m[15], 0xfe2ce6e0u, 10);
    MD5_STEP(MD5_I, c, d, a, b, m[6], 0xa3014314u, 15);
    MD5_STEP(MD5_I, b, c, d, a, m[13], 0x4e0811a1u, 21);
    MD5_STEP(MD5_I, a, b, c, d, m[4], 0xf7537e82u, 6);
    MD5_STEP(MD5_I, d, a, b, c, m[11], 0xbd3af235u, 10);
    MD5_STEP(MD5_I, c, d, a, b, m[2], 0x2ad7d2bbu, 15);
    MD5_STEP(MD5_I, b, c, d, a, m[9], 0xeb86d391u, 21);
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
}

// 16 bytes at p; aligned -> one dwordx4, otherwise byte loads.
__device__ __forceinline__ uint4 load16(const uint8_t *p, bool aligned)
{
    if (aligned)
        return *reinterpret_cast<const uint4 *>(p);
    uint32_t w[4];
#pragma unroll
    for (int d = 0; d < 4; d++)
        w[d] = (uint32_t)p[4 * d] | ((uint32_t)p[4 * d + 1] << 8) |
               ((uint32_t)p[4 * d + 2] << 16) | ((uint32_t)p[4 * d + 3] << 24);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void store_sig(uint8_t *sig, uint64_t L, uint32_t w2, uint32_t w3,
                                          uint32_t w4, uint32_t w5)
{
    uint2 *sp = reinterpret_cast<uint2 *>(sig);
    sp[0] = make_uint2(bswap32((uint32_t)(L >> 32)), bswap32((uint32_t)L));
    sp[1] = make_uint2(w2, w3);
    sp[2] = make_uint2(w4, w5);
}

// Final block(s) of a file whose first nblk full 64-byte blocks are already
// folded into st: the L & 63 tail bytes, 0x80, zero pad and the 64-bit bit
// length (RFC 1321 3.1-3.2; my_md5_final at storage/storage_dio.c:512).
__device__ __forceinline__ void md5_finish(uint32_t st[4], const uint8_t *p, uint64_t nblk,
                                           uint64_t L)
{
    const uint8_t *tp = p + (nblk << 6);
    const uint32_t r = (uint32_t)(L & 63u);
    uint32_t m[16];
#pragma unroll
    for (int wd = 0; wd < 16; wd++) {
        uint32_t word = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t k = 4 * wd + q;
            uint32_t b = 0;
            if (k < r) {
                b = tp[k];
            } else if (k == r) {
                b = 0x80u;
            }
            word |= b << (8 * q);
        }
        m[wd] = word;
    }
    const uint64_t bits = L << 3;
    if (r < 56) {
        m[14] = (uint32_t)bits;
        m[15] = (uint32_t)(bits >> 32);
        md5_compress(st, m);
    } else {
        md5_compress(st, m);
#pragma unroll
        for (int wd = 0; wd < 14; wd++)
            m[wd] = 0;
        m[14] = (uint32_t)bits;
        m[15] = (uint32_t)(bits >> 32);
        md5_compress(st, m);
    }
}

// ------------------------------------------------------- lane-per-file path

// One 16-byte vector through all four CALC_HASH_CODES4 hashes.
// PL: simple_hash / Time33 as 16-byte polynomial steps on v_dot4_u32_u8
// (poly16_step) instead of byte-serial shift-adds; ELF stays byte-serial.
template <bool SAR, bool NP, bool PL>
__device__ __forceinline__ void h4_vec(const uint32_t *sD, uint32_t lb, uint32_t K16, uint4 q,
                                       uint32_t &c, uint32_t &e, uint32_t &s, uint32_t &t)
{
    if constexpr (NP)
        c = chain16p<SAR>(sD, lb, c, q, K16);
    else
        c = chain16<SAR>(sD, c, q, K16);
    if constexpr (PL) {
        elf_word<SAR>(q.x, e);
        elf_word<SAR>(q.y, e);
        elf_word<SAR>(q.z, e);
        elf_word<SAR>(q.w, e);
        s = poly16_step<31>(s, q);
        t = poly16_step<33>(t, q);
    } else {
        h3_word<SAR>(q.x, e, s, t);
        h3_word<SAR>(q.y, e, s, t);
        h3_word<SAR>(q.z, e, s, t);
        h3_word<SAR>(q.w, e, s, t);
    }
}

// The same with the CRC through the conflict-free rotated slice-by-8 tables.
template <bool SAR, bool PL>
__device__ __forceinline__ void h4_vec_r(const uint32_t *sR, const Rep8Lane &R, uint32_t K8,
                                         uint4 q, uint32_t &c, uint32_t &e, uint32_t &s,
                                         uint32_t &t)
{
    c = chain16r<SAR>(sR, R, c, q, K8);
    elf_word<SAR>(q.x, e);
    elf_word<SAR>(q.y, e);
    elf_word<SAR>(q.z, e);
    elf_word<SAR>(q.w, e);
    s = poly16_step<31>(s, q);
    t = poly16_step<33>(t, q);
}

constexpr int kLaneBlock7 = 768;

template <bool SAR, int METHOD, int VAR>
__global__ __launch_bounds__(VAR == 4 ? 1024 : (VAR == 7 ? kLaneBlock7 : 256), VAR == 6 ? 8 : 1) void sig_lane_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint64_t *__restrict__ sizes, const uint32_t *__restrict__ order, uint32_t n,
    const DevTables *__restrict__ tabs, uint32_t *__restrict__ crc_out,
    uint8_t *__restrict__ sig_out, int32_t *__restrict__ codes_out)
{
    // VAR 4: the VAR 2 load schedule with the CRC through the conflict-free
    // v_perm nibble tables (64 KiB of LDS) instead of 8-bit slice tables.
    constexpr bool NP = (VAR == 4);
    constexpr bool RP = (VAR == 7);  // rotated replicated slice-by-8 CRC tables
    constexpr bool PL = (VAR == 5 || VAR == 6 || VAR == 7);  // VAR 6: VAR 5 capped at 64 VGPRs
    __shared__ uint32_t sD[NP ? kNibPDwords : (RP ? kRep8Dwords : 16 * 256)];
    __shared__ uint32_t sT[256];
    if constexpr (METHOD == 1) {  // the MD5 path uses no tables
        if constexpr (NP)
            lds_fill_nibp(sD, &tabs->N[0][0]);
        else if constexpr (RP)
            lds_fill_rep8(sD, &tabs->t.D[0][0]);
        else
            lds_fill(sD, &tabs->t.D[0][0], 16 * 256);
        lds_fill(sT, tabs->t.T, 256);
        __syncthreads();
    }

    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t lb = (threadIdx.x & 31) * 4u;
    const uint32_t K16 = RP ? tabs->t.K8 : tabs->t.K16;
    const Rep8Lane R8 = rep8_lane(threadIdx.x & 63);
    const uint32_t f = order ? order[i] : i;
    const uint64_t L = sizes[f];
    const uint8_t *p = base + offs[f];
    uint32_t c = 0xFFFFFFFFu;  // CRC32_XINIT (storage/storage_service.c:7149)

    if (METHOD == 1) {
        uint32_t e = 0, s = 0, t = 0;  // INIT_HASH_CODES4 (storage/storage_service.c:7156)
        uint64_t head = (16u - ((uintptr_t)p & 15u)) & 15u;
        if (head > L)
            head = L;
        for (uint64_t k = 0; k < head; k++) {
            const uint32_t b = p[k];
            c = crc_byte<SAR>(sT, c, b);
            h3_byte<SAR>(b, e, s, t);
        }
#define H4V(Q, C, E, S, T)                                      \
    do {                                                        \
        if constexpr (RP)                                       \
            h4_vec_r<SAR, PL>(sD, R8, K16, (Q), C, E, S, T);     \
        else                                                    \
            h4_vec<SAR, NP, PL>(sD, lb, K16, (Q), C, E, S, T);   \
    } while (0)
        const uint4 *v = reinterpret_cast<const uint4 *>(p + head);
        const uint64_t nvec = (L - head) >> 4;
        uint64_t j = 0;
        if constexpr (VAR == 0) {
            if (nvec) {
                // 16 B per step, loads running 3 vectors ahead (the index is
                // clamped so the tail re-reads the last vector: no
                // conditional loads in the loop).
                const uint64_t last = nvec - 1;
                uint4 q0 = v[0];
                uint4 q1 = v[last < 1 ? last : 1];
                uint4 q2 = v[last < 2 ? last : 2];
                for (; j < nvec; j++) {
                    const uint64_t nj = j + 3;
                    const uint4 q3 = v[nj < last ? nj : last];
                    H4V(q0, c, e, s, t);
                    q0 = q1;
                    q1 = q2;
                    q2 = q3;
                }
            }
        } else if constexpr (VAR == 1) {
            // 64 B per step, the next 64 B loaded while this one is hashed
            if (nvec >= 4) {
                uint4 a0 = v[0], a1 = v[1], a2 = v[2], a3 = v[3];
                for (; j + 4 <= nvec; j += 4) {
                    const uint64_t nx = (j + 8 <= nvec) ? j + 4 : j;
                    const uint4 b0 = v[nx], b1 = v[nx + 1], b2 = v[nx + 2], b3 = v[nx + 3];
                    H4V(a0, c, e, s, t);
                    H4V(a1, c, e, s, t);
                    H4V(a2, c, e, s, t);
                    H4V(a3, c, e, s, t);
                    a0 = b0;
                    a1 = b1;
                    a2 = b2;
                    a3 = b3;
                }
            }
        } else if constexpr (VAR == 3) {
            // 64 B per step, no register prefetch (fewer VGPRs, more waves)
            for (; j + 4 <= nvec; j += 4) {
                uint4 a[4];
#pragma unroll
                for (int q = 0; q < 4; q++)
                    a[q] = v[j + q];
#pragma unroll
                for (int q = 0; q < 4; q++)
                    H4V(a[q], c, e, s, t);
            }
        } else {
            // 128 B (one cache line) per step, no register prefetch.  Single
            // vectors first until the window is 128-byte aligned, so every
            // step reads exactly one whole line (an unaligned window splits
            // two lines across steps, and the second touch misses L2).
            const uint64_t lead = ((128u - ((uintptr_t)v & 127u)) & 127u) >> 4;
            for (; j < lead && j < nvec; j++)
                H4V( v[j], c, e, s, t);
            for (; j + 8 <= nvec; j += 8) {
                uint4 a[8];
#pragma unroll
                for (int q = 0; q < 8; q++)
                    a[q] = v[j + q];
#pragma unroll
                for (int q = 0; q < 8; q++)
                    H4V(a[q], c, e, s, t);
            }
        }
        for (; j < nvec; j++)
            H4V(v[j], c, e, s, t);
        for (uint64_t k = head + (nvec << 4); k < L; k++) {
            const uint32_t b = p[k];
            c = crc_byte<SAR>(sT, c, b);
            h3_byte<SAR>(b, e, s, t);
        }
#undef H4V
        c ^= 0xFFFFFFFFu;  // CRC32_FINAL / FINISH_HASH_CODES4 (storage/storage_dio.c:500,508)
        crc_out[f] = c;
        if (sig_out)
            store_sig(sig_out + 24ull * f, L, bswap32(c), bswap32(e), bswap32(s), bswap32(t));
        if (codes_out)
            reinterpret_cast<int4 *>(codes_out)[f] = make_int4((int)c, (int)e, (int)s, (int)t);
    } else {
        uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};  // my_md5_init
        const bool al = (((uintptr_t)p) & 15u) == 0;
        const uint64_t nblk = L >> 6;
        uint64_t j = 0;
        // MD5 only: the file CRC of the MD5 method comes from crc_seg_kernel
        // on a forked stream (launch_sig_lane).  A lane-serial CRC here put
        // LDS-latency waits into the in-order MD5 chain of a wave that has
        // no partner wave to hide them (1-2 waves per SIMD at 1-4 MiB files).
        auto md5_block = [&](uint4 a0, uint4 a1, uint4 a2, uint4 a3) {
            const uint32_t m[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                                    a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
            md5_compress(st, m);
        };
        if (al) {
            // The MD5 chain is serial per file, and a batch of 1-4 MiB files
            // leaves ~1-2 waves per SIMD: deep register prefetch (the next
            // 4 blocks load while 4 are hashed) hides HBM latency instead.
            // hipcc sinks ordinary prefetch loads to their use (it re-issues
            // invariant loads instead of keeping 64 VGPRs live), so the next
            // group is loaded with asm loads that it cannot move, and waited
            // for by one asm wait that names every destination.
            const uint4 *v = reinterpret_cast<const uint4 *>(p);
            constexpr int G = 4;
            if (nblk >= G) {
                uint4 A[4 * G];
#pragma unroll
                for (int q = 0; q < 4 * G; q++)
                    A[q] = v[q];
                for (; j + G <= nblk; j += G) {
                    const uint64_t nx = (j + 2 * G <= nblk) ? j + G : j;
                    const uint4 *np = v + 4 * nx;
                    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                    u32x4 b0, b1, b2, b3, b4, b5, b6, b7, b8, b9, b10, b11, b12, b13, b14, b15;
#define MD5_PF(x, q) asm volatile("global_load_dwordx4 %0, %1, off offset:%2" \
                                  : "=v"(x) : "v"(np), "i"(16 * (q)) : "memory")
                    MD5_PF(b0, 0); MD5_PF(b1, 1); MD5_PF(b2, 2); MD5_PF(b3, 3);
                    MD5_PF(b4, 4); MD5_PF(b5, 5); MD5_PF(b6, 6); MD5_PF(b7, 7);
                    MD5_PF(b8, 8); MD5_PF(b9, 9); MD5_PF(b10, 10); MD5_PF(b11, 11);
                    MD5_PF(b12, 12); MD5_PF(b13, 13); MD5_PF(b14, 14); MD5_PF(b15, 15);
#undef MD5_PF
#pragma unroll
                    for (int b = 0; b < G; b++)
                        md5_block(A[4 * b], A[4 * b + 1], A[4 * b + 2], A[4 * b + 3]);
                    asm volatile("s_waitcnt vmcnt(0)"
                                 : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3) :: "memory");
                    asm volatile("" : "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7));
                    asm volatile("" : "+v"(b8), "+v"(b9), "+v"(b10), "+v"(b11));
                    asm volatile("" : "+v"(b12), "+v"(b13), "+v"(b14), "+v"(b15));
#define MD5_MV(q) A[q] = make_uint4(b##q[0], b##q[1], b##q[2], b##q[3])
                    MD5_MV(0); MD5_MV(1); MD5_MV(2); MD5_MV(3);
                    MD5_MV(4); MD5_MV(5); MD5_MV(6); MD5_MV(7);
                    MD5_MV(8); MD5_MV(9); MD5_MV(10); MD5_MV(11);
                    MD5_MV(12); MD5_MV(13); MD5_MV(14); MD5_MV(15);
#undef MD5_MV
                }
            }
            for (; j < nblk; j++)
                md5_block(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
        } else if (nblk) {
            uint4 a0 = load16(p, al), a1 = load16(p + 16, al), a2 = load16(p + 32, al),
                  a3 = load16(p + 48, al);
            for (; j < nblk; j++) {
                const uint8_t *q = p + ((j + 1 < nblk) ? (j + 1) : j) * 64;
                const uint4 b0 = load16(q, al), b1 = load16(q + 16, al), b2 = load16(q + 32, al),
                            b3 = load16(q + 48, al);
                const uint32_t m[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                                        a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
                md5_compress(st, m);
                a0 = b0;
                a1 = b1;
                a2 = b2;
                a3 = b3;
            }
        }
        md5_finish(st, p, nblk, L);
        if (sig_out)  // memcpy(sig + 8, md5 digest, 16) (storage/storage_service.c:119)
            store_sig(sig_out + 24ull * f, L, st[0], st[1], st[2], st[3]);
        if (codes_out)
            reinterpret_cast<int4 *>(codes_out)[f] =
                make_int4((int)st[0], (int)st[1], (int)st[2], (int)st[3]);
    }
}

// ------------------------------------------------ MD5 path, staged loads
//
// MD5 is serial per file, so it stays one LANE per file, but the bytes do not
// travel lane-per-file.  A lane-per-file load touches 64 files (64 pages) per
// wave-instruction; over a batch of 100K 1-4 MiB files that is ~100K
// concurrently open pages and the address translation, not the MD5 chain or
// HBM, set the time.  Here each round the wave loads
// CH bytes of each of its 64 files cooperatively: every load instruction
// reads whole 256-byte runs of 4 files (16 lanes x 16 B each), the data is
// written to LDS as one padded row per file, and each lane then hashes its
// own row.  The next round's loads are in flight (asm, so hipcc cannot sink
// them to their use) while this round is hashed.
//
// LDS row stride CH+16: ds_write_b128 groups (8 lanes = 128 contiguous bytes
// of one row) and ds_read_b128 groups (16 lanes, rows l..l+15 at quad
// (l + const) mod 16) are both conflict-free.
constexpr int kMd5Chunk = 256;

template <int CH>
__global__ __launch_bounds__(64) void md5_stage_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint64_t *__restrict__ sizes, const uint32_t *__restrict__ order, uint32_t n,
    const uint8_t *__restrict__ safe, uint8_t *__restrict__ sig_out, int32_t *__restrict__ codes_out)
{
    constexpr int PIECES = CH / 16;   // 16-byte pieces of one file's chunk
    constexpr int FPI = 64 / PIECES;  // files per load instruction
    constexpr int NLD = 64 / FPI;     // load instructions per round
    constexpr int STRIDE = CH + 16;   // padded LDS row per file
    constexpr int BPR = CH / 64;      // MD5 blocks per round
    static_assert(CH == 256 && NLD == 16, "the asm wait below names 16 registers");
    __shared__ __attribute__((aligned(16))) uint8_t sbuf[64 * STRIDE];
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

    const int lane = threadIdx.x;
    const uint32_t i = blockIdx.x * 64 + lane;
    const bool valid = i < n;
    const uint32_t f = valid ? order[i] : 0;
    const uint64_t L = valid ? sizes[f] : 0;
    const uint8_t *p = valid ? base + offs[f] : safe;
    const uint64_t nblk = L >> 6;
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};  // my_md5_init

    if (__all((((uintptr_t)p) & 15u) == 0)) {
        uint64_t mx = nblk;
#pragma unroll
        for (int o = 32; o; o >>= 1) {
            const uint64_t y = __shfl_xor(mx, o);
            mx = y > mx ? y : mx;
        }
        const uint64_t rounds = (mx + BPR - 1) / BPR;
        const int piece = lane % PIECES, fsub = lane / PIECES;
        const uint8_t *lp[NLD];
        uint32_t lim[NLD];  // valid 16-byte pieces (full blocks) of the loaded file
#pragma unroll
        for (int k = 0; k < NLD; k++) {
            const int src = k * FPI + fsub;
            lp[k] = reinterpret_cast<const uint8_t *>(__shfl((uintptr_t)p, src)) + piece * 16;
            const uint64_t nb = __shfl(nblk, src);
            lim[k] = nb >= (1ull << 30) ? 0xFFFFFFFFu : (uint32_t)(nb * 4);
        }
        u32x4 R[NLD];
        auto issue = [&](uint64_t r) {
            const uint32_t rp = (uint32_t)r * PIECES + piece;
            const uint64_t roff = r * CH;
#pragma unroll
            for (int k = 0; k < NLD; k++) {
                const uint8_t *a = (rp < lim[k]) ? lp[k] + roff : safe;
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(R[k]) : "v"(a) : "memory");
            }
        };
        if (rounds)
            issue(0);
        const uint8_t *mine = sbuf + lane * STRIDE;
        for (uint64_t r = 0; r < rounds; r++) {
            __syncthreads();  // the previous round's row reads precede these writes
            asm volatile("s_waitcnt vmcnt(0)"
                         : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]), "+v"(R[4]), "+v"(R[5]),
                           "+v"(R[6]), "+v"(R[7]), "+v"(R[8]), "+v"(R[9]), "+v"(R[10]),
                           "+v"(R[11]), "+v"(R[12]), "+v"(R[13]), "+v"(R[14]), "+v"(R[15])
                         :: "memory");
#pragma unroll
            for (int k = 0; k < NLD; k++)
                *reinterpret_cast<u32x4 *>(sbuf + (k * FPI + fsub) * STRIDE + piece * 16) = R[k];
            __syncthreads();
            if (r + 1 < rounds)
                issue(r + 1);
#pragma unroll
            for (int b = 0; b < BPR; b++) {
                if (r * BPR + b < nblk) {
                    const uint4 *q = reinterpret_cast<const uint4 *>(mine + b * 64);
                    const uint4 a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
                    const uint32_t m[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                                            a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
                    md5_compress(st, m);
                }
            }
        }
    } else {
        // some file of this wave starts off a 16-byte boundary: lane-serial
        // byte-assembled loads (rare; bulk-ingest batches are aligned)
        for (uint64_t j = 0; j < nblk; j++) {
            const uint8_t *q = p + j * 64;
            const uint4 a0 = load16(q, false), a1 = load16(q + 16, false),
                        a2 = load16(q + 32, false), a3 = load16(q + 48, false);
            const uint32_t m[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                                    a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
            md5_compress(st, m);
        }
    }
    if (!valid)
        return;
    md5_finish(st, p, nblk, L);
    if (sig_out)  // memcpy(sig + 8, md5 digest, 16) (storage/storage_service.c:119)
        store_sig(sig_out + 24ull * f, L, st[0], st[1], st[2], st[3]);
    if (codes_out)
        reinterpret_cast<int4 *>(codes_out)[f] =
            make_int4((int)st[0], (int)st[1], (int)st[2], (int)st[3]);
}

// ------------------------------------------------------- segmented CRC path

// 0xFF in every byte of the dword at byte offset `off` that lies in [lo, hi).
__device__ __forceinline__ uint32_t byte_range_mask(int64_t off, int64_t lo, int64_t hi)
{
    const int64_t a = lo - off < 0 ? 0 : lo - off;
    const int64_t b = hi - off > 4 ? 4 : hi - off;
    if (b <= a)
        return 0;
    const uint32_t upto_b = b >= 4 ? 0xFFFFFFFFu : ((1u << (8 * b)) - 1u);
    const uint32_t upto_a = (1u << (8 * a)) - 1u;  // a < 4 here
    return upto_b & ~upto_a;
}

// First vector(s) of a segment: bytes before the segment start (offset a0)
// become the neutral byte (0xFF in the complemented SAR domain, 0 otherwise);
// for the unsigned variant the file's bytes 0..3 are XOR 0xFF (the XINIT
// identity, DESIGN.md "K2 segmented CRC").
template <bool SAR>
__device__ __forceinline__ uint4 seg_fix_vector(uint4 w, int64_t off, int64_t a0, bool xor4)
{
    uint32_t d[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int64_t o = off + 4 * k;
        const uint32_t inv = byte_range_mask(o, INT64_MIN / 2, a0);
        d[k] = SAR ? (d[k] | inv) : (d[k] & ~inv);
        if (!SAR && xor4)
            d[k] ^= byte_range_mask(o, a0, a0 + 4);
    }
    return make_uint4(d[0], d[1], d[2], d[3]);
}

// Zero-init CRC state of the (masked) bytes [Ap, Ap+len) of one segment,
// computed by the whole wave.  Vectors are 16-byte aligned in memory and the
// 4 KiB block grid is aligned to the segment's last full vector, so the only
// partial vector is the first (leading neutral bytes do not change a
// zero-init state).  See DESIGN.md "K2 segmented CRC" for the algebra.
// Table modes of the segmented kernel: 0 = 8-bit slice-by-16 (16 KiB),
// 1 = nibble tables (64 KiB, v_perm addressed), 2 = rotated replicated
// slice-by-8 (64 KiB, conflict-free; K is then K8).
template <bool SAR, int TM>
__device__ __forceinline__ uint32_t chain16x(const uint32_t *sD, uint32_t lb, const Rep8Lane &R,
                                             uint32_t c, uint4 w, uint32_t K)
{
    if constexpr (TM == 1)
        return chain16p<SAR>(sD, lb, c, w, K);
    else if constexpr (TM == 2)
        return chain16r<SAR>(sD, R, c, w, K);
    else
        return chain16<SAR>(sD, c, w, K);
}

template <bool SAR, int TM>
__device__ __forceinline__ uint32_t crc_segment(const uint32_t *sD, const uint32_t *sT,
                                                const uint32_t *sA, const uint32_t *sR,
                                                const Rep8Lane &R8, uint32_t K16,
                                                const uint8_t *Ap, uint64_t len, bool first_seg,
                                                int lane)
{
    const uint32_t lb = (uint32_t)(lane & 31) * 4u;
    const int64_t a0 = (int64_t)((uintptr_t)Ap & 15u);  // segment start within its vector
    const uint4 *v = reinterpret_cast<const uint4 *>(Ap - a0);
    const int64_t e_off = a0 + (int64_t)len;
    const int64_t nvec = e_off >> 4;  // full vectors ending at or before the end
    const bool xor4 = !SAR && first_seg;
    uint32_t state = 0;
    if (nvec > 0) {
        const int64_t J = (nvec + 255) >> 8;
        const uint4 neutral = SAR ? make_uint4(~0u, ~0u, ~0u, ~0u) : make_uint4(0, 0, 0, 0);
        uint32_t acc = 0;
        {  // first (partial) block: vectors before index 0 are neutral
            const int64_t vb = nvec - 256 * J + 4 * lane;
            uint4 w[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int64_t vi = vb + q;
                w[q] = v[vi < 0 ? 0 : vi];
                if (vi < 0)
                    w[q] = neutral;
                else if (16 * vi < a0 + 4)
                    w[q] = seg_fix_vector<SAR>(w[q], 16 * vi, a0, xor4);
            }
#pragma unroll
            for (int q = 0; q < 4; q++)
                acc = chain16x<SAR, TM>(sD, lb, R8, acc, w[q], K16);
        }
        // blocks 1..J-1: the next block's 64 B per lane is loaded while this
        // one is folded (index clamped on the last block: no branch)
        uint4 nx[4];
        if (J > 1) {
            const uint4 *vp = v + (nvec - 256 * (J - 1) + 4 * lane);
#pragma unroll
            for (int q = 0; q < 4; q++)
                nx[q] = vp[q];
        }
        for (int64_t jb = 1; jb < J; jb++) {
            uint4 w[4];
#pragma unroll
            for (int q = 0; q < 4; q++)
                w[q] = nx[q];
            const int64_t jn = (jb + 1 < J) ? jb + 1 : jb;
            const uint4 *vp = v + (nvec - 256 * (J - jn) + 4 * lane);
#pragma unroll
            for (int q = 0; q < 4; q++)
                nx[q] = vp[q];
            acc = apply4(sA, acc);  // advance 4032 B to this lane's next piece
            if (jb == 1 && nvec - 256 * (J - 1) == 1 && lane == 0)
                w[0] = seg_fix_vector<SAR>(w[0], 16, a0, xor4);  // vector 1 opens block 1
#pragma unroll
            for (int q = 0; q < 4; q++)
                acc = chain16x<SAR, TM>(sD, lb, R8, acc, w[q], K16);
        }
        // wave reduction: lane group values relative to the group's end
#pragma unroll
        for (int lv = 0; lv < 6; lv++) {
            const uint32_t u = apply4(sR + lv * 1024, acc);
            const uint32_t o = __shfl_xor(u, 1 << lv);
            if (lane & (1 << lv))
                acc ^= o;
        }
        state = __shfl(acc, 63);
    }
    const int64_t t0 = (16 * nvec > a0) ? 16 * nvec : a0;
    for (int64_t o = t0; o < e_off; o++) {
        uint32_t b = Ap[o - a0];
        if (SAR || (xor4 && o < a0 + 4))
            b ^= 0xFFu;
        state = crc_byte<SAR>(sT, state, b);
    }
    return state;
}

static_assert(kSegBytes == 65536, "CrcTables::ADVSEG is built for 64 KiB segments");

// Advance state v by n zero bytes (v -> M^n v) with the GF(2) matrix powers
// M^(2^k): lane c (< 32) holds column c, one 5-step XOR reduction per set
// bit of n.  Wave-uniform v and n; returns the advanced state in every lane.
__device__ __forceinline__ uint32_t advance_any(const DevTables *__restrict__ tabs, uint32_t v,
                                                uint64_t n, int lane)
{
    const int col = lane & 31;
    for (int kk = 0; n; kk++, n >>= 1) {
        if (!(n & 1))
            continue;
        uint32_t part = ((v >> col) & 1u) ? tabs->t.MPOW[kk][col] : 0u;
        part ^= __shfl_xor(part, 16);
        part ^= __shfl_xor(part, 8);
        part ^= __shfl_xor(part, 4);
        part ^= __shfl_xor(part, 2);
        part ^= __shfl_xor(part, 1);
        v = part;
    }
    return v;
}

// Constant making crc0(masked data) into CRC32_FINAL(CRC32_ex(data, XINIT)).
template <bool SAR>
__device__ __forceinline__ uint32_t crc_final_const(uint64_t L)
{
    if (SAR)
        return 0;
    return 0xFFFFFFFFu ^ (L < 4 ? (0xFFFFFFFFu >> (8 * (uint32_t)L)) : 0u);
}

template <bool SAR, int TM>
__global__ __launch_bounds__(kSegBlock) void crc_seg_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint64_t *__restrict__ sizes, const uint64_t *__restrict__ seg_first, uint32_t n,
    const DevTables *__restrict__ tabs, uint32_t *__restrict__ crc_out)
{
    // TM 1/2 (64 KiB conflict-free tables): the reduction tables stay in
    // global memory (24 lookups per segment).  TM 0: everything in LDS.
    constexpr int kD = TM == 1 ? kNibPDwords : (TM == 2 ? kRep8Dwords : 16 * 256);
    constexpr int kR = TM ? 0 : 6 * 4 * 256;
    __shared__ uint32_t smem[kD + 256 + 2 * 4 * 256 + kR];
    uint32_t *sD = smem, *sT = smem + kD, *sA = sT + 256, *sS = sA + 1024;
    const uint32_t *sR = TM ? &tabs->t.ADVRED[0][0][0] : sS + 1024;
    lds_fill(sS, &tabs->t.ADVSEG[0][0], 4 * 256);
    if constexpr (TM == 1)
        lds_fill_nibp(sD, SAR ? &tabs->Nc[0][0] : &tabs->N[0][0]);
    else if constexpr (TM == 2)
        lds_fill_rep8(sD, SAR ? &tabs->Dc[0][0] : &tabs->t.D[0][0]);
    else
        lds_fill(sD, SAR ? &tabs->Dc[0][0] : &tabs->t.D[0][0], 16 * 256);
    lds_fill(sT, tabs->t.T, 256);
    lds_fill(sA, &tabs->t.ADV4032[0][0], 4 * 256);
    if constexpr (!TM)
        lds_fill(sS + 1024, &tabs->t.ADVRED[0][0][0], 6 * 4 * 256);
    __syncthreads();

    const uint32_t K16 = TM == 2 ? tabs->t.K8 : tabs->t.K16;
    const Rep8Lane R8 = rep8_lane(threadIdx.x & 63);
    const int lane = threadIdx.x & 63;
    const uint64_t wpb = blockDim.x >> 6;
    const uint64_t w = (uint64_t)blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * wpb;
    const uint64_t total = seg_first[n];
    uint64_t s = (total * w) / nw;
    const uint64_t s_end = (total * (w + 1)) / nw;
    if (s >= s_end)
        return;
    uint32_t lo = 0, hi = n;  // last f with seg_first[f] <= s
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (seg_first[mid] <= s)
            lo = mid;
        else
            hi = mid;
    }
    uint32_t f = lo;
    // The wave's segments are consecutive, so a run of segments of one file
    // is chained in place (state = ADV_seg(state) ^ crc0(seg), one 4-lookup
    // advance per segment); only when the run ends is the state advanced to
    // the file end (GF(2) matrix powers) and merged into crc_out.
    uint32_t run_f = 0xFFFFFFFFu, run_state = 0;
    uint64_t run_end = 0;
    bool run_has_first = false, run_whole = false;
    for (;; s++) {
        const bool more = s < s_end;
        if (more) {
            while (seg_first[f + 1] <= s)
                f++;
        }
        if (run_f != 0xFFFFFFFFu && (!more || f != run_f)) {  // flush the finished run
            const uint64_t L = sizes[run_f];
            const uint32_t cl = run_has_first ? crc_final_const<SAR>(L) : 0u;
            if (run_whole) {
                if (lane == 0)
                    crc_out[run_f] = run_state ^ cl;
            } else {
                const uint32_t v = advance_any(tabs, run_state, L - run_end, lane);
                if (lane == 0)
                    atomicXor(&crc_out[run_f], v ^ cl);
            }
            run_f = 0xFFFFFFFFu;
        }
        if (!more)
            break;
        const uint64_t k = s - seg_first[f];
        const uint64_t nseg = seg_first[f + 1] - seg_first[f];
        const uint64_t L = sizes[f];
        const uint8_t *fp = base + offs[f];
        const uint64_t lo_b = k * kSegBytes;
        const uint64_t hi_b = (L < lo_b + kSegBytes) ? L : lo_b + kSegBytes;
        const uint32_t v = crc_segment<SAR, TM>(sD, sT, sA, sR, R8, K16, fp + lo_b, hi_b - lo_b, k == 0, lane);
        if (run_f == f) {
            const uint64_t len = hi_b - lo_b;
            const uint32_t adv = (len == kSegBytes) ? apply4(sS, run_state)
                                                    : advance_any(tabs, run_state, len, lane);
            run_state = adv ^ v;
        } else {
            run_f = f;
            run_state = v;
            run_has_first = (k == 0);
        }
        run_end = hi_b;
        run_whole = run_has_first && (k + 1 == nseg);
    }
}

// ---------------------------------------------------------------- planning

__global__ void plan_nseg_kernel(const uint64_t *__restrict__ sizes, uint32_t n,
                                 uint64_t *__restrict__ nseg, uint32_t *__restrict__ crc_out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t L = sizes[i];
    nseg[i] = (L + kSegBytes - 1) / kSegBytes;
    crc_out[i] = 0;  // empty files keep CRC 0; multi-segment files accumulate by XOR
}

__device__ __forceinline__ uint32_t size_bin(uint64_t L)
{
    if (L == 0)
        return 0;
    const uint32_t e = 63 - __builtin_clzll(L);
    const uint32_t m = (e >= 5) ? (uint32_t)((L >> (e - 5)) & 31u) : (uint32_t)((L << (5 - e)) & 31u);
    return e * 32 + m;  // < kSizeBins
}

__global__ void bin_hist_kernel(const uint64_t *__restrict__ sizes, uint32_t n,
                                uint32_t *__restrict__ hist)
{
    __shared__ uint32_t h[kSizeBins];
    for (int b = threadIdx.x; b < kSizeBins; b += blockDim.x)
        h[b] = 0;
    __syncthreads();
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        atomicAdd(&h[size_bin(sizes[i])], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < kSizeBins; b += blockDim.x)
        if (h[b])
            atomicAdd(&hist[b], h[b]);
}

// Descending exclusive scan of the bin histogram (one block of kSizeBins threads / 2).
__global__ __launch_bounds__(1024) void bin_scan_kernel(const uint32_t *__restrict__ hist,
                                                        uint32_t *__restrict__ cursor)
{
    __shared__ uint32_t s[kSizeBins];
    for (int b = threadIdx.x; b < kSizeBins; b += blockDim.x)
        s[b] = hist[kSizeBins - 1 - b];  // reversed: largest bin first
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int b = 0; b < kSizeBins; b++) {
            const uint32_t c = s[b];
            s[b] = run;
            run += c;
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kSizeBins; b += blockDim.x)
        cursor[kSizeBins - 1 - b] = s[b];
}

__global__ __launch_bounds__(1024) void bin_scatter_kernel(const uint64_t *__restrict__ sizes,
                                                           uint32_t n, uint32_t *__restrict__ cursor,
                                                           uint32_t *__restrict__ order)
{
    __shared__ uint32_t cnt[kSizeBins];
    __shared__ uint32_t bas[kSizeBins];
    for (int b = threadIdx.x; b < kSizeBins; b += blockDim.x)
        cnt[b] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t bin = 0, rank = 0;
    if (i < n) {
        bin = size_bin(sizes[i]);
        rank = atomicAdd(&cnt[bin], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kSizeBins; b += blockDim.x)
        if (cnt[b])
            bas[b] = atomicAdd(&cursor[b], cnt[b]);
    __syncthreads();
    if (i < n)
        order[bas[bin] + rank] = i;
}

// -------------------------------------------------------- exclusive scan u64

constexpr int kScanBlock = 256;
constexpr int kScanItems = 4;
constexpr int kScanTile = kScanBlock * kScanItems;

__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t *wsum, uint64_t &total)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= o)
            x += y;
    }
    if (lane == 63)
        wsum[wid] = x;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); k++) {
        if (k < wid)
            pre += wsum[k];
        tot += wsum[k];
    }
    __syncthreads();
    total = tot;
    return pre + x - v;
}

__global__ __launch_bounds__(kScanBlock) void scan_reduce_kernel(const uint64_t *__restrict__ in,
                                                                 uint64_t n,
                                                                 uint64_t *__restrict__ bsum)
{
    __shared__ uint64_t wsum[kScanBlock / 64];
    const uint64_t b0 = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; k++)
        if (b0 + k < n)
            v += in[b0 + k];
    uint64_t tot;
    block_exclusive_scan(v, wsum, tot);
    if (threadIdx.x == 0)
        bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanBlock) void scan_sums_kernel(uint64_t *__restrict__ bsum,
                                                               uint64_t nb)
{
    __shared__ uint64_t wsum[kScanBlock / 64];
    uint64_t carry = 0;
    for (uint64_t c0 = 0; c0 < nb; c0 += kScanBlock) {
        const uint64_t i = c0 + threadIdx.x;
        const uint64_t v = (i < nb) ? bsum[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_exclusive_scan(v, wsum, tot);
        if (i < nb)
            bsum[i] = carry + ex;
        carry += tot;
    }
}

__global__ __launch_bounds__(kScanBlock) void scan_apply_kernel(const uint64_t *__restrict__ in,
                                                                uint64_t n,
                                                                const uint64_t *__restrict__ bsum,
                                                                uint64_t *__restrict__ out)
{
    __shared__ uint64_t wsum[kScanBlock / 64];
    const uint64_t b0 = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint64_t vals[kScanItems];
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        vals[k] = (b0 + k < n) ? in[b0 + k] : 0;
        v += vals[k];
    }
    uint64_t tot;
    uint64_t run = bsum[blockIdx.x] + block_exclusive_scan(v, wsum, tot);
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        if (b0 + k < n)
            out[b0 + k] = run;
        run += vals[k];
    }
    if (b0 < n && b0 + kScanItems >= n)  // the thread holding the last element writes the total
        out[n] = run;
}

// ------------------------------------------------------------------ launchers

hipError_t launch_exclusive_scan(const uint64_t *in, uint64_t n, uint64_t *out, uint64_t *bsum,
                                 hipStream_t st)
{
    if (n == 0)
        return hipMemsetAsync(out, 0, sizeof(uint64_t), st);
    const uint64_t nb = (n + kScanTile - 1) / kScanTile;
    scan_reduce_kernel<<<(unsigned)nb, kScanBlock, 0, st>>>(in, n, bsum);
    scan_sums_kernel<<<1, kScanBlock, 0, st>>>(bsum, nb);
    scan_apply_kernel<<<(unsigned)nb, kScanBlock, 0, st>>>(in, n, bsum, out);
    return hipGetLastError();
}

uint64_t scan_workspace_elems(uint64_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

hipError_t launch_sig_lane(bool sar, int method, const uint8_t *base, const uint64_t *offs,
                           const uint64_t *sizes, uint32_t n, uint32_t *hist, uint32_t *order,
                           const DevTables *tabs, uint32_t *crc_out, uint8_t *sig_out,
                           int32_t *codes_out, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1)
{
    hipError_t e = hipMemsetAsync(hist, 0, sizeof(uint32_t) * kSizeBins * 2, st);
    if (e != hipSuccess)
        return e;
    uint32_t *cursor = hist + kSizeBins;
    const unsigned hb = (n + 1023) / 1024;
    bin_hist_kernel<<<hb < 1024 ? hb : 1024, 256, 0, st>>>(sizes, n, hist);
    bin_scan_kernel<<<1, 1024, 0, st>>>(hist, cursor);
    bin_scatter_kernel<<<hb, 1024, 0, st>>>(sizes, n, cursor, order);
    const unsigned g = (n + 255) / 256, g4 = (n + 1023) / 1024;
    if (ev0)
        (void)hipEventRecord(ev0, st);
    const unsigned g7 = (n + kLaneBlock7 - 1) / kLaneBlock7;
#define LANE_LAUNCH(S, M, V) \
    sig_lane_kernel<S, M, V><<<(V == 4) ? g4 : ((V == 7) ? g7 : g), (V == 4) ? 1024 : ((V == 7) ? kLaneBlock7 : 256), 0, st>>>( \
        base, offs, sizes, order, n, tabs, crc_out, sig_out, codes_out)
    static int var = -1;
    if (var < 0) {  // FDFS_GPU_LANE_VARIANT: A/B of the hash-path load schedule
        const char *ev = getenv("FDFS_GPU_LANE_VARIANT");
        var = ev ? (ev[0] - '0') : 5;
        if (var != 2 && var != 6 && var != 7)
            var = 5;
    }
    static int md5v = -1;
    if (md5v < 0) {  // FDFS_GPU_MD5_LANE=1: the lane-per-file load path (A/B only)
        const char *ev = getenv("FDFS_GPU_MD5_LANE");
        md5v = (ev && ev[0] == '1') ? 1 : 0;
    }
    if (method == 2 && md5v == 0) {
        md5_stage_kernel<kMd5Chunk><<<(n + 63) / 64, 64, 0, st>>>(
            base, offs, sizes, order, n, reinterpret_cast<const uint8_t *>(tabs), sig_out,
            codes_out);
    } else if (method == 2) {
        if (sar)
            LANE_LAUNCH(true, 2, 0);
        else
            LANE_LAUNCH(false, 2, 0);
    } else if (sar) {
        if (var == 7)
            LANE_LAUNCH(true, 1, 7);
        else if (var == 5)
            LANE_LAUNCH(true, 1, 5);
        else if (var == 6)
            LANE_LAUNCH(true, 1, 6);
        else
            LANE_LAUNCH(true, 1, 2);
    } else {
        if (var == 7)
            LANE_LAUNCH(false, 1, 7);
        else if (var == 5)
            LANE_LAUNCH(false, 1, 5);
        else if (var == 6)
            LANE_LAUNCH(false, 1, 6);
        else
            LANE_LAUNCH(false, 1, 2);
    }
#undef LANE_LAUNCH
    if (ev1)
        (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

hipError_t launch_crc_seg(bool sar, const uint8_t *base, const uint64_t *offs, const uint64_t *sizes,
                          uint32_t n, uint64_t *nseg, uint64_t *seg_first, uint64_t *bsum,
                          const DevTables *tabs, uint32_t *crc_out, unsigned grid, hipStream_t st,
                          hipEvent_t ev0, hipEvent_t ev1)
{
    plan_nseg_kernel<<<(n + 255) / 256, 256, 0, st>>>(sizes, n, nseg, crc_out);
    hipError_t e = launch_exclusive_scan(nseg, n, seg_first, bsum, st);
    if (e != hipSuccess)
        return e;
    if (ev0)
        (void)hipEventRecord(ev0, st);
    const int tm = crc_table_mode();
#define SEG_LAUNCH(S, T) \
    crc_seg_kernel<S, T><<<grid, kSegBlock, 0, st>>>(base, offs, sizes, seg_first, n, tabs, crc_out)
    if (sar) {
        if (tm == 2)
            SEG_LAUNCH(true, 2);
        else if (tm == 1)
            SEG_LAUNCH(true, 1);
        else
            SEG_LAUNCH(true, 0);
    } else {
        if (tm == 2)
            SEG_LAUNCH(false, 2);
        else if (tm == 1)
            SEG_LAUNCH(false, 1);
        else
            SEG_LAUNCH(false, 0);
    }
#undef SEG_LAUNCH
    if (ev1)
        (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

// Table form of the segmented CRC kernel: FDFS_GPU_CRC_TABLES = rep8
// (default, conflict-free), nib, or byte (A/B measurement only).
int crc_table_mode()
{
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("FDFS_GPU_CRC_TABLES");
        v = (e && e[0] == 'n') ? 1 : ((e && e[0] == 'b') ? 0 : 2);
    }
    return v;
}

int crc_seg_blocks_per_cu()
{
    int nb = 0;
    const int tm = crc_table_mode();
    hipError_t e = tm == 2   ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, crc_seg_kernel<true, 2>, kSegBlock, 0)
                   : tm == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, crc_seg_kernel<true, 1>, kSegBlock, 0)
                             : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, crc_seg_kernel<true, 0>, kSegBlock, 0);
    if (e != hipSuccess)
        return 1;
    return nb > 0 ? nb : 1;
}

}  // namespace fdfs
