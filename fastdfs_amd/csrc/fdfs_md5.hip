// MD5 signature path (FDFS_SIG_MD5, file_signature_method=md5; config 3).
//
// Reference: my_md5_init / my_md5_update / my_md5_final (libfastcommon md5.c,
// RSA RFC 1321 code) driven by storage/storage_dio.c:480,512 and initialised
// at storage/storage_service.c:7160; the digest is the signature tail
// (storage/storage_service.c:106-120).
#include "fdfs_device.hpp"
#include "fdfs_kernels.hpp"

#include <cstdlib>

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
#define MD5_H(b, c, d) ((b) ^ (c) ^ (d))
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

// ------------------------------------------------ MD5 path, staged loads
//
// MD5 is serial per file, so it stays one LANE per file, but the bytes do not
// travel lane-per-file.  A lane-per-file load touches 64 files (64 pages) per
// wave-instruction; over a batch of 100K 1-4 MiB files that is ~100K
// concurrently open pages and the address translation, not the MD5 chain or
// HBM, set the time.  Here each round the wave loads
// CH bytes of each of its 64 files cooperatively: every load instruction
// reads whole 128-byte lines of 8 files (8 lanes x 16 B each), the data is
// written to LDS as one padded row per file, and each lane then hashes its
// own row.  The next round's loads are in flight while this round is hashed
// (two register sets, asm loads so hipcc cannot sink them to their use).
//
// The file's CRC32 (CRC32_ex over the same bytes, storage/storage_dio.c:467)
// is computed by the same lane from the same LDS row: one pass over HBM for
// CRC + MD5.  Its table lookups are independent of the MD5 chain, so they
// fill the issue slots a latency-bound MD5 wave leaves empty.  The slice-by-16
// tables are shared by the workgroup's waves (waves are otherwise
// independent: no barrier after the table fill).
//
// LDS row stride CH+16 = 144 B: ds_write_b128 groups (8 lanes = one 128-byte
// row) and ds_read_b128 groups (16 lanes, rows f at quad 9f + const mod 16)
// are both conflict-free.
constexpr int kMd5Chunk = 128;
constexpr int kMd5Waves = 4;

template <bool SAR>
__global__ __launch_bounds__(64 * kMd5Waves) void md5_stage_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint64_t *__restrict__ sizes, const uint32_t *__restrict__ order, uint32_t n,
    const DevTables *__restrict__ tabs, uint32_t w1, uint32_t *__restrict__ queue,
    uint32_t *__restrict__ crc_out, uint8_t *__restrict__ sig_out, int32_t *__restrict__ codes_out)
{
    constexpr int CH = kMd5Chunk;
    constexpr int PIECES = CH / 16;   // 16-byte pieces of one file's chunk
    constexpr int FPI = 64 / PIECES;  // files per load instruction
    constexpr int NLD = 64 / FPI;     // load instructions per round
    constexpr int STRIDE = CH + 16;   // padded LDS row per file
    constexpr int BPR = CH / 64;      // MD5 blocks per round
    static_assert(NLD == 8, "the asm waits below name 8 registers");
    __shared__ uint32_t sD[16 * 256];
    __shared__ uint32_t sT[256];
    __shared__ __attribute__((aligned(16))) uint8_t sbuf[kMd5Waves][64 * STRIDE];
    lds_fill(sD, &tabs->t.D[0][0], 16 * 256);
    lds_fill(sT, tabs->t.T, 256);
    __syncthreads();
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

    const int lane = threadIdx.x & 63;
    // Waves take 64-file chunks of the size-descending order.  Every wave is
    // resident at once (a few per SIMD), so the kernel ends with the SIMD
    // that holds the most bytes: the first `w1` waves (one workgroup per
    // CU) take the largest chunks and the rest take the remaining chunks
    // smallest first, so a CU's second workgroup is a light one.
    //
    // With a queue (the default) the grid is one workgroup per CU, one wave
    // per SIMD, and each wave takes the next chunk from a device counter
    // until none is left: the first chunks taken are the largest, and the
    // rest go to the waves whose chunks end first, so small files run in the
    // time the largest ones take instead of beside them (fewer files stream
    // at once while the longest chains run).
    const uint32_t nw = (n + 63) / 64;
    uint8_t *tile = sbuf[threadIdx.x >> 6];
    const uint8_t *safe = reinterpret_cast<const uint8_t *>(tabs);  // >= 16 readable bytes
    const uint32_t K16 = tabs->t.K16;
    uint32_t chunk;
    if (queue) {
        uint32_t c0 = 0;
        if (lane == 0)
            c0 = atomicAdd(queue, 1u);
        chunk = __shfl(c0, 0);
    } else {
        const uint32_t w = blockIdx.x * kMd5Waves + (threadIdx.x >> 6);
        chunk = (w < w1) ? w : nw - 1 - (w - w1);
        if (w >= nw)
            chunk = nw;
    }
    for (; chunk < nw;) {
    const uint32_t wave0 = chunk * 64;
    const uint32_t i = wave0 + lane;
    const bool valid = i < n;
    const uint32_t f = valid ? order[i] : 0;
    const uint64_t L = valid ? sizes[f] : 0;
    const uint8_t *p = valid ? base + offs[f] : safe;
    const uint64_t nblk = L >> 6;
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};  // my_md5_init
    uint32_t c = 0xFFFFFFFFu;  // CRC32_XINIT (storage/storage_service.c:7149)

    auto block = [&](uint4 a0, uint4 a1, uint4 a2, uint4 a3) {
        const uint32_t m[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                                a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
        md5_compress(st, m);
        c = chain16<SAR>(sD, c, a0, K16);
        c = chain16<SAR>(sD, c, a1, K16);
        c = chain16<SAR>(sD, c, a2, K16);
        c = chain16<SAR>(sD, c, a3, K16);
    };

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
        uint64_t lim[NLD];  // 16-byte pieces in the loaded file's full blocks
#pragma unroll
        for (int k = 0; k < NLD; k++) {
            const int src = k * FPI + fsub;
            lp[k] = reinterpret_cast<const uint8_t *>(__shfl((uintptr_t)p, src)) + piece * 16;
            lim[k] = __shfl(nblk, src) * 4;
        }
        u32x4 RA[NLD], RB[NLD];
        auto issue = [&](u32x4 (&R)[NLD], uint64_t r) {  // unconditional: past the end reads `safe`
            const uint64_t rp = r * PIECES + piece;
#pragma unroll
            for (int k = 0; k < NLD; k++) {
                const uint8_t *a = (rp < lim[k]) ? lp[k] + r * CH : safe;
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(R[k]) : "v"(a) : "memory");
            }
        };
        auto stage = [&](u32x4 (&R)[NLD]) {  // R = the older of two sets in flight
            asm volatile("s_waitcnt vmcnt(8)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]) :: "memory");
            asm volatile("" : "+v"(R[4]), "+v"(R[5]), "+v"(R[6]), "+v"(R[7]));
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = 0; k < NLD; k++)
                *reinterpret_cast<u32x4 *>(tile + (k * FPI + fsub) * STRIDE + piece * 16) = R[k];
            __builtin_amdgcn_wave_barrier();
        };
        const uint8_t *mine = tile + lane * STRIDE;
        auto hash_round = [&](uint64_t r) {
#pragma unroll
            for (int b = 0; b < BPR; b++) {
                if (r * BPR + b < nblk) {
                    const uint4 *q = reinterpret_cast<const uint4 *>(mine + b * 64);
                    block(q[0], q[1], q[2], q[3]);
                }
            }
            __builtin_amdgcn_wave_barrier();
        };
        issue(RA, 0);
        for (uint64_t r = 0; r < rounds; r += 2) {
            issue(RB, r + 1);
            stage(RA);
            hash_round(r);
            issue(RA, r + 2);
            stage(RB);
            if (r + 1 < rounds)
                hash_round(r + 1);
        }
        asm volatile("s_waitcnt vmcnt(0)"
                     : "+v"(RA[0]), "+v"(RA[1]), "+v"(RA[2]), "+v"(RA[3]), "+v"(RA[4]), "+v"(RA[5]),
                       "+v"(RA[6]), "+v"(RA[7]) :: "memory");
    } else {
        // some file of this wave starts off a 16-byte boundary: lane-serial
        // byte-assembled loads (rare; bulk-ingest batches are aligned)
        for (uint64_t j = 0; j < nblk; j++) {
            const uint8_t *q = p + j * 64;
            block(load16(q, false), load16(q + 16, false), load16(q + 32, false), load16(q + 48, false));
        }
    }
    if (valid) {
        for (uint64_t k = nblk << 6; k < L; k++)  // CRC of the L & 63 tail bytes
            c = crc_byte<SAR>(sT, c, p[k]);
        md5_finish(st, p, nblk, L);
        crc_out[f] = c ^ 0xFFFFFFFFu;  // CRC32_FINAL (storage/storage_dio.c:500)
        if (sig_out)  // memcpy(sig + 8, md5 digest, 16) (storage/storage_service.c:119)
            store_sig(sig_out + 24ull * f, L, st[0], st[1], st[2], st[3]);
        if (codes_out)
            reinterpret_cast<int4 *>(codes_out)[f] =
                make_int4((int)st[0], (int)st[1], (int)st[2], (int)st[3]);
    }
    if (!queue)
        break;
    uint32_t c1 = 0;
    if (lane == 0)
        c1 = atomicAdd(queue, 1u);
    chunk = __shfl(c1, 0);
    }
}

hipError_t launch_md5_stage(bool sar, const uint8_t *base, const uint64_t *offs,
                            const uint64_t *sizes, uint32_t n, const uint32_t *order,
                            const DevTables *tabs, uint32_t *queue, uint32_t *crc_out, uint8_t *sig_out,
                            int32_t *codes_out, hipStream_t st)
{
    static int ncu[64];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess)
        return e;
    if (dev < 0 || dev >= 64)
        return hipErrorInvalidDevice;
    if (ncu[dev] == 0 &&
        (e = hipDeviceGetAttribute(&ncu[dev], hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess)
        return e;
#ifdef FDFS_PROBES
    static int mode = -1;
    if (mode < 0) {  // A/B (make probes): FDFS_GPU_MD5_QUEUE=0 -> one chunk per wave, all resident
        const char *ev = getenv("FDFS_GPU_MD5_QUEUE");
        mode = ev ? atoi(ev) : 1;
    }
#else
    constexpr int mode = 1;
#endif
    constexpr unsigned kBlk = 64 * kMd5Waves;
    const uint32_t nw = (n + 63) / 64;
    unsigned grid = (n + kBlk - 1) / kBlk;
    uint32_t *q = nullptr;
    if (mode && queue) {  // queue zeroed by the caller (launch_sig_lane's workspace memset)
        q = queue;
        const unsigned g = (unsigned)ncu[dev];
        grid = g < (nw + kMd5Waves - 1) / kMd5Waves ? g : (nw + kMd5Waves - 1) / kMd5Waves;
    }
    const uint32_t w1 = (uint32_t)ncu[dev] * kMd5Waves;
    if (sar)
        md5_stage_kernel<true><<<grid, kBlk, 0, st>>>(base, offs, sizes, order, n, tabs, w1, q, crc_out,
                                                      sig_out, codes_out);
    else
        md5_stage_kernel<false><<<grid, kBlk, 0, st>>>(base, offs, sizes, order, n, tabs, w1, q, crc_out,
                                                       sig_out, codes_out);
    return hipGetLastError();
}

}  // namespace fdfs
