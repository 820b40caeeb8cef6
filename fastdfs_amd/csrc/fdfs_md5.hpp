// RFC 1321 MD5 compression (the my_md5_* arithmetic of libfastcommon md5.c,
// storage/storage_dio.c:480,512), shared by the lane kernels and the
// chunked-update finaliser.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#ifndef MD5_CHAIN_ASM
#define MD5_CHAIN_ASM 1
#endif

namespace fdfs {

// ----------------------------------------------------------------- MD5 core

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s)
{
    return __builtin_amdgcn_alignbit(x, x, 32 - s);
}

#define MD5_F(b, c, d) ((d) ^ ((b) & ((c) ^ (d))))
#define MD5_G(b, c, d) ((c) ^ ((d) & ((b) ^ (c))))
#define MD5_H(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0x96)  // one op, not two v_xor
#define MD5_I(b, c, d) ((c) ^ ((b) | ~(d)))
// The step's critical path is F -> add -> rotate -> add.  a, m and k are
// known steps ahead, so (a + m + k) is summed off the path and the on-path
// add is kept a single full-rate v_add_u32 (hipcc would otherwise fold it
// into a v_add3_u32, a half-rate instruction on the chain).
__device__ __forceinline__ uint32_t add_chain(uint32_t x, uint32_t y)
{
#if MD5_CHAIN_ASM
    uint32_t r;
    asm("v_add_u32_e32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
#else
    return x + y;
#endif
}
#define MD5_STEP(FN, a, b, c, d, m, k, s) a = (b) + rotl(add_chain((a) + (m) + (k), FN(b, c, d)), s)

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

// One round (16 steps) of a block whose K[i] + m[g(i)] sums were made in
// advance (md5_chain_wg's helper wave): q[u] holds steps 16 R + 4 u .. + 3.
// With the sum given, the step is four dependent VALU (F, v_add3_u32,
// rotate, add) and nothing off the chain: on one wave alone on its SIMD, 16.8
// against 21.2 cycles per byte for md5_compress (profiles/r06/chain_lds_ubench.json).
#define MD5_KSTEP(FN, a, b, c, d, km, s) a = (b) + rotl((a) + (km) + FN(b, c, d), s)
template <int R>
__device__ __forceinline__ void md5_round_km(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, const uint4 q[4])
{
    constexpr int S[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
#pragma unroll
    for (int u = 0; u < 4; u++) {
        if constexpr (R == 0) {
            MD5_KSTEP(MD5_F, a, b, c, d, q[u].x, S[R][0]);
            MD5_KSTEP(MD5_F, d, a, b, c, q[u].y, S[R][1]);
            MD5_KSTEP(MD5_F, c, d, a, b, q[u].z, S[R][2]);
            MD5_KSTEP(MD5_F, b, c, d, a, q[u].w, S[R][3]);
        } else if constexpr (R == 1) {
            MD5_KSTEP(MD5_G, a, b, c, d, q[u].x, S[R][0]);
            MD5_KSTEP(MD5_G, d, a, b, c, q[u].y, S[R][1]);
            MD5_KSTEP(MD5_G, c, d, a, b, q[u].z, S[R][2]);
            MD5_KSTEP(MD5_G, b, c, d, a, q[u].w, S[R][3]);
        } else if constexpr (R == 2) {
            MD5_KSTEP(MD5_H, a, b, c, d, q[u].x, S[R][0]);
            MD5_KSTEP(MD5_H, d, a, b, c, q[u].y, S[R][1]);
            MD5_KSTEP(MD5_H, c, d, a, b, q[u].z, S[R][2]);
            MD5_KSTEP(MD5_H, b, c, d, a, q[u].w, S[R][3]);
        } else {
            MD5_KSTEP(MD5_I, a, b, c, d, q[u].x, S[R][0]);
            MD5_KSTEP(MD5_I, d, a, b, c, q[u].y, S[R][1]);
            MD5_KSTEP(MD5_I, c, d, a, b, q[u].z, S[R][2]);
            MD5_KSTEP(MD5_I, b, c, d, a, q[u].w, S[R][3]);
        }
    }
}
#undef MD5_KSTEP

// The final block(s) after the L & 63 pending bytes (RFC 1321 3.1-3.2):
// m holds those bytes (any value past them); 0x80, zero pad and the 64-bit
// bit count are put in and one or two blocks compressed.
__device__ __forceinline__ void md5_pad_compress(uint32_t st[4], uint32_t m[16], uint32_t r,
                                                 uint32_t bits_lo, uint32_t bits_hi)
{
#pragma unroll
    for (int wd = 0; wd < 16; wd++) {
        const int vb = (int)r - 4 * wd;  // pending bytes in this word
        uint32_t w = vb >= 4 ? m[wd] : (vb <= 0 ? 0u : (m[wd] & ((1u << (8 * vb)) - 1u)));
        if (vb >= 0 && vb < 4)
            w |= 0x80u << (8 * vb);
        m[wd] = w;
    }
    if (r >= 56) {
        md5_compress(st, m);
#pragma unroll
        for (int wd = 0; wd < 14; wd++)
            m[wd] = 0;
    }
    m[14] = bits_lo;
    m[15] = bits_hi;
    md5_compress(st, m);
}

}  // namespace fdfs
