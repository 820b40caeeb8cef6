// Microbenchmark: can a single byte-serial chain (one big file's ELFHash_ex
// or MD5, one lane of one wave alone on its SIMD) run faster when a helper
// wave prepares its operands?  The chain wave issues at most one VALU per ~4
// cycles, so off-chain work in the chain wave (the ELF byte extraction, the
// MD5 a + m + k sum) costs the chain issue slots.
//   elfc   the shipped 3-op chain form with in-wave byte extraction (chain_ubench's elfc)
//   elfb   the same chain on bytes already one per dword (no extraction)
//   elfl   elfb with the byte-dwords read from an LDS ring (ds_read_b128) that a
//          helper wave of the same workgroup fills from HBM (the candidate kernel)
//   md5    fdfs_md5.hpp md5_compress (5 VALU per step, a + m + k off the chain)
//   md5k   K + m summed in advance, v_add3_u32 on the chain (4 VALU per step)
//   md5l   md5k with K + m read from an LDS ring a helper wave fills from HBM
// One workgroup per CU (W = 1: one chain wave per CU).  Cycles from s_memtime,
// the clock from s_memrealtime.
// Build: hipcc -O3 --offload-arch=gfx950 -I../../fastdfs_amd/csrc chain_lds_ubench.hip -o chain_lds_ubench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "fdfs_device.hpp"
#include "fdfs_md5.hpp"

using namespace fdfs;

struct Stamp {
    unsigned long long c0, c1, t0, t1;
};

__device__ __forceinline__ void elf_b(uint32_t b, uint32_t &e, uint32_t &y)
{
    const uint32_t t = (e << 4) + b;
    y = (uint32_t)((int32_t)t >> 24);
    e = t ^ (y & 0xFFFFFFF0u);
}

__global__ void k_elfc(int iters, const uint8_t *, uint32_t *out, Stamp *st)
{
    if (threadIdx.x >= 64)
        return;
    uint32_t e = threadIdx.x, y = 0;
    uint32_t w0 = threadIdx.x * 0x9E3779B9u, w1 = w0 ^ 0x85EBCA6Bu, w2 = w0 + 0xC2B2AE35u, w3 = ~w0;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
        elf_word4_chain<true, false>(w0, e);
        elf_word4_chain<true, false>(w1, e);
        elf_word4_chain<true, false>(w2, e);
        elf_word4_chain_y<true>(w3, e, y);
        w0 += e;
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 64 + threadIdx.x] = e ^ y;
    if (threadIdx.x == 0)
        st[blockIdx.x] = Stamp{c0, c1, t0, t1};
}

__global__ void k_elfb(int iters, const uint8_t *, uint32_t *out, Stamp *st)
{
    if (threadIdx.x >= 64)
        return;
    uint32_t e = threadIdx.x, y = 0;
    uint32_t b[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
        b[k] = (threadIdx.x * 0x9E3779B9u >> k) & 0xFFu;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++)
            elf_b(b[k], e, y);
        b[0] = (b[0] + e) & 0xFFu;
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 64 + threadIdx.x] = e ^ y;
    if (threadIdx.x == 0)
        st[blockIdx.x] = Stamp{c0, c1, t0, t1};
}

constexpr uint32_t kSlot = 4096;  // file bytes per LDS slot (16 KiB of byte-dwords)
constexpr uint32_t kSrc = 1u << 20;  // bytes each workgroup streams per pass

// wave 0: the chain over the byte-dwords of slot k; wave 1: fills slot k + 1.
__global__ __launch_bounds__(128) void k_elfl(int iters, const uint8_t *src, uint32_t *out, Stamp *st)
{
    __shared__ uint4 ring[2][kSlot / 4];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint8_t *p = src + (size_t)blockIdx.x * kSrc;
    const uint32_t nslots = (uint32_t)iters;  // slots of kSlot bytes (wrapping over kSrc)
    auto fill = [&](int s, uint32_t k) {
        const uint8_t *q = p + (size_t)(k * kSlot) % kSrc;
        uint32_t *r = reinterpret_cast<uint32_t *>(ring[s]);
#pragma unroll 4
        for (int j = 0; j < (int)(kSlot / 64); j += 16) {
            uint32_t v[16];
#pragma unroll
            for (int u = 0; u < 16; u++)
                v[u] = q[(j + u) * 64 + lane];
#pragma unroll
            for (int u = 0; u < 16; u++)
                r[(j + u) * 64 + lane] = v[u];
        }
    };
    uint32_t e = 0, y = 0;
    unsigned long long c0 = 0, t0 = 0;
    if (wv == 1)
        fill(0, 0);
    else {
        __builtin_amdgcn_s_setprio(3);
        c0 = __builtin_amdgcn_s_memtime();
        t0 = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    for (uint32_t k = 0; k < nslots; k++) {
        if (wv == 1) {
            if (k + 1 < nslots)
                fill((k + 1) & 1, k + 1);
        } else {
            const uint4 *r = ring[k & 1];
            uint4 a = r[0], b = r[1], c = r[2], d = r[3];
            for (uint32_t g = 0; g < kSlot / 16; g++) {
                const uint32_t gn = (g + 1) & (kSlot / 16 - 1);
                const uint4 na = r[4 * gn], nb = r[4 * gn + 1], nc = r[4 * gn + 2], nd = r[4 * gn + 3];
                elf_b(a.x, e, y); elf_b(a.y, e, y); elf_b(a.z, e, y); elf_b(a.w, e, y);
                elf_b(b.x, e, y); elf_b(b.y, e, y); elf_b(b.z, e, y); elf_b(b.w, e, y);
                elf_b(c.x, e, y); elf_b(c.y, e, y); elf_b(c.z, e, y); elf_b(c.w, e, y);
                elf_b(d.x, e, y); elf_b(d.y, e, y); elf_b(d.z, e, y); elf_b(d.w, e, y);
                a = na; b = nb; c = nc; d = nd;
            }
        }
        __syncthreads();
    }
    if (wv == 0) {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
        out[blockIdx.x * 64 + lane] = e ^ y;
        if (lane == 0)
            st[blockIdx.x] = Stamp{c0, c1, t0, t1};
    }
}

__global__ void k_md5(int iters, const uint8_t *, uint32_t *out, Stamp *st)
{
    if (threadIdx.x >= 64)
        return;
    uint32_t s[4] = {0x67452301u ^ threadIdx.x, 0xefcdab89u, 0x98badcfeu, 0x10325476u ^ blockIdx.x};
    uint32_t m[16];
#pragma unroll
    for (int k = 0; k < 16; k++)
        m[k] = (threadIdx.x * 0x9E3779B9u) ^ (k * 0x85EBCA6Bu) ^ blockIdx.x;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
        md5_compress(s, m);
        m[i & 15] ^= s[0];
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 64 + threadIdx.x] = s[0] ^ s[1] ^ s[2] ^ s[3];
    if (threadIdx.x == 0)
        st[blockIdx.x] = Stamp{c0, c1, t0, t1};
}

// MD5 with km[i] = K[i] + m[g(i)] given: a = b + rotl(a + km + F, s), the
// three-input sum one v_add3_u32 on the chain.
__constant__ uint32_t kMd5K[64] = {
    0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u, 0xfd469501u,
    0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u, 0xa679438eu, 0x49b40821u,
    0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du, 0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u,
    0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu, 0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au,
    0xfffa3942u, 0x8771f681u, 0x6d9d6122u, 0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u,
    0x289b7ec6u, 0xeaa127fau, 0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u,
    0xf4292244u, 0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,
    0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu, 0xeb86d391u};
__host__ __device__ constexpr int md5_g(int i)
{
    return i < 16 ? i : i < 32 ? (5 * i + 1) & 15 : i < 48 ? (3 * i + 5) & 15 : (7 * i) & 15;
}
__host__ __device__ constexpr int md5_s(int i)
{
    constexpr int S[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
    return S[(i >> 4) * 4 + (i & 3)];
}
#define MD5_KSTEP(FN, a, b, c, d, km, s) a = (b) + rotl((a) + (km) + FN(b, c, d), s)

template <typename KM>
__device__ __forceinline__ void md5_compress_km(uint32_t st[4], KM &&km)
{
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#pragma unroll
    for (int i = 0; i < 64; i += 4) {
        const int r = i >> 4;
        if (r == 0) {
            MD5_KSTEP(MD5_F, a, b, c, d, km(i), md5_s(i));
            MD5_KSTEP(MD5_F, d, a, b, c, km(i + 1), md5_s(i + 1));
            MD5_KSTEP(MD5_F, c, d, a, b, km(i + 2), md5_s(i + 2));
            MD5_KSTEP(MD5_F, b, c, d, a, km(i + 3), md5_s(i + 3));
        } else if (r == 1) {
            MD5_KSTEP(MD5_G, a, b, c, d, km(i), md5_s(i));
            MD5_KSTEP(MD5_G, d, a, b, c, km(i + 1), md5_s(i + 1));
            MD5_KSTEP(MD5_G, c, d, a, b, km(i + 2), md5_s(i + 2));
            MD5_KSTEP(MD5_G, b, c, d, a, km(i + 3), md5_s(i + 3));
        } else if (r == 2) {
            MD5_KSTEP(MD5_H, a, b, c, d, km(i), md5_s(i));
            MD5_KSTEP(MD5_H, d, a, b, c, km(i + 1), md5_s(i + 1));
            MD5_KSTEP(MD5_H, c, d, a, b, km(i + 2), md5_s(i + 2));
            MD5_KSTEP(MD5_H, b, c, d, a, km(i + 3), md5_s(i + 3));
        } else {
            MD5_KSTEP(MD5_I, a, b, c, d, km(i), md5_s(i));
            MD5_KSTEP(MD5_I, d, a, b, c, km(i + 1), md5_s(i + 1));
            MD5_KSTEP(MD5_I, c, d, a, b, km(i + 2), md5_s(i + 2));
            MD5_KSTEP(MD5_I, b, c, d, a, km(i + 3), md5_s(i + 3));
        }
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
}

__global__ void k_md5k(int iters, const uint8_t *, uint32_t *out, Stamp *st)
{
    if (threadIdx.x >= 64)
        return;
    uint32_t s[4] = {0x67452301u ^ threadIdx.x, 0xefcdab89u, 0x98badcfeu, 0x10325476u ^ blockIdx.x};
    uint32_t km[64];
#pragma unroll
    for (int k = 0; k < 64; k++)
        km[k] = (threadIdx.x * 0x9E3779B9u) ^ (k * 0x85EBCA6Bu) ^ blockIdx.x;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
        md5_compress_km(s, [&](int j) { return km[j]; });
        km[0] ^= s[0];
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 64 + threadIdx.x] = s[0] ^ s[1] ^ s[2] ^ s[3];
    if (threadIdx.x == 0)
        st[blockIdx.x] = Stamp{c0, c1, t0, t1};
}

constexpr uint32_t kMBlocks = 64;  // MD5 blocks per LDS slot (16 KiB of K + m)

// wave 0: MD5 over slot k's K + m words; wave 1: lane i computes step i's
// K[i] + m[g(i)] of each block of slot k + 1.
__global__ __launch_bounds__(128) void k_md5l(int iters, const uint8_t *src, uint32_t *out, Stamp *st)
{
    __shared__ uint4 ring[2][kMBlocks * 16];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t *p = reinterpret_cast<const uint32_t *>(src + (size_t)blockIdx.x * kSrc);
    const uint32_t nslots = (uint32_t)iters;
    const uint32_t kk = kMd5K[lane];
    const int g = md5_g(lane);
    auto fill = [&](int s, uint32_t k) {
        const uint32_t *q = p + ((size_t)k * kMBlocks * 16) % (kSrc / 4);
        uint32_t *r = reinterpret_cast<uint32_t *>(ring[s]);
#pragma unroll 4
        for (int j = 0; j < (int)kMBlocks; j += 16) {
            uint32_t v[16];
#pragma unroll
            for (int u = 0; u < 16; u++)
                v[u] = q[(j + u) * 16 + g];
#pragma unroll
            for (int u = 0; u < 16; u++)
                r[(j + u) * 64 + lane] = v[u] + kk;
        }
    };
    uint32_t s[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    unsigned long long c0 = 0, t0 = 0;
    if (wv == 1)
        fill(0, 0);
    else {
        __builtin_amdgcn_s_setprio(3);
        c0 = __builtin_amdgcn_s_memtime();
        t0 = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    for (uint32_t k = 0; k < nslots; k++) {
        if (wv == 1) {
            if (k + 1 < nslots)
                fill((k + 1) & 1, k + 1);
        } else {
            const uint4 *r = ring[k & 1];
            for (uint32_t blk = 0; blk < kMBlocks; blk++) {
                uint4 w[16];
#pragma unroll
                for (int u = 0; u < 16; u++)
                    w[u] = r[blk * 16 + u];
                md5_compress_km(s, [&](int j) {
                    const uint4 &x = w[j >> 2];
                    return (j & 3) == 0 ? x.x : (j & 3) == 1 ? x.y : (j & 3) == 2 ? x.z : x.w;
                });
            }
        }
        __syncthreads();
    }
    if (wv == 0) {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
        out[blockIdx.x * 64 + lane] = s[0] ^ s[1] ^ s[2] ^ s[3];
        if (lane == 0)
            st[blockIdx.x] = Stamp{c0, c1, t0, t1};
    }
}

int main()
{
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *out;
    uint8_t *src;
    Stamp *st, *hst;
    hipMalloc(&out, sizeof(uint32_t) * 64 * ncu);
    hipMalloc(&st, sizeof(Stamp) * ncu);
    hipMalloc(&src, (size_t)kSrc * ncu);
    hipMemset(src, 0x5A, (size_t)kSrc * ncu);
    hst = new Stamp[ncu];
    printf("{\"cus\": %d, \"runs\": [\n", ncu);
    struct K {
        const char *name;
        void (*fn)(int, const uint8_t *, uint32_t *, Stamp *);
        int iters, block;
        double bytes_per_iter;
    };
    const K ks[] = {{"elfc", k_elfc, 20000, 64, 16.0},     {"elfb", k_elfb, 20000, 64, 16.0},
                    {"elfl", k_elfl, 80, 128, (double)kSlot}, {"md5", k_md5, 4000, 64, 64.0},
                    {"md5k", k_md5k, 4000, 64, 64.0},       {"md5l", k_md5l, 64, 128, 64.0 * kMBlocks}};
    bool first = true;
    for (const K &k : ks) {
        for (int rep = 0; rep < 2; rep++) {
            hipLaunchKernelGGL(k.fn, dim3(ncu), dim3(k.block), 0, 0, k.iters, src, out, st);
            hipDeviceSynchronize();
        }
        hipMemcpy(hst, st, sizeof(Stamp) * ncu, hipMemcpyDeviceToHost);
        double cyc = 0, ns = 0;
        for (int b = 0; b < ncu; b++) {
            cyc += (double)(hst[b].c1 - hst[b].c0);
            ns += (double)(hst[b].t1 - hst[b].t0) * 10.0;
        }
        cyc /= ncu;
        ns /= ncu;
        const double per_byte = cyc / (k.iters * k.bytes_per_iter);
        printf("%s{\"kernel\": \"%s\", \"cycles_per_byte_lane\": %.4f, \"clock_ghz\": %.3f, \"ns\": %.0f}",
               first ? "" : ",\n", k.name, per_byte, cyc / ns, ns);
        first = false;
    }
    printf("\n]}\n");
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
