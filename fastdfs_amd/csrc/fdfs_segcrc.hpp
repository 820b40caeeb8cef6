// Segment-parallel CRC32_ex building blocks (device side) of crc_seg_kernel
// (fdfs_sig.hip).  Reference loop:
// storage/storage_dio.c:465-467 (CRC32_ex over each chunk).
#pragma once
#include "fdfs_device.hpp"
#include "fdfs_kernels.hpp"

namespace fdfs {

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
// The tables are the rotated, replicated slice-by-8 form (64 KiB,
// conflict-free; fdfs_device.hpp chain16r), with K = K8.
template <bool SAR>
__device__ __forceinline__ uint32_t crc_segment(const uint32_t *sD, const uint32_t *sT,
                                                const uint32_t *sA, const uint32_t *sR,
                                                const Rep8Lane &R8, uint32_t K8,
                                                const uint8_t *Ap, uint64_t len, bool first_seg,
                                                int lane)
{
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
        // lane `lane` folds vectors 4 lane .. 4 lane + 3 of each 4 KiB block
        auto lidx = [&](int64_t blk0, int q) -> int64_t { return blk0 + 4 * lane + q; };
        uint4 nx[4];
        {  // first (partial) block: vectors before index 0 are neutral
            const int64_t b0 = nvec - 256 * J;
            const int64_t vb = b0 + 4 * lane;
            uint4 w[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int64_t li = lidx(b0, q);
                w[q] = v[li < 0 ? 0 : li];
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int64_t vi = vb + q;
                if (vi < 0)
                    w[q] = neutral;
                else if (16 * vi < a0 + 4)
                    w[q] = seg_fix_vector<SAR>(w[q], 16 * vi, a0, xor4);
            }
#pragma unroll
            for (int q = 0; q < 4; q++)
                acc = chain16r<SAR>(sD, R8, acc, w[q], K8);
        }
        // blocks 1..J-1: the next block's 64 B per lane is loaded while this
        // one is folded (index clamped on the last block: no branch)
        if (J > 1) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                nx[q] = v[lidx(nvec - 256 * (J - 1), q)];
        }
        for (int64_t jb = 1; jb < J; jb++) {
            uint4 w[4];
#pragma unroll
            for (int q = 0; q < 4; q++)
                w[q] = nx[q];
            {
                const int64_t jn = (jb + 1 < J) ? jb + 1 : jb;
#pragma unroll
                for (int q = 0; q < 4; q++)
                    nx[q] = v[lidx(nvec - 256 * (J - jn), q)];
            }
            acc = apply4(sA, acc);  // advance 4032 B to this lane's next piece
            if (jb == 1 && nvec - 256 * (J - 1) == 1 && lane == 0)
                w[0] = seg_fix_vector<SAR>(w[0], 16, a0, xor4);  // vector 1 opens block 1
#pragma unroll
            for (int q = 0; q < 4; q++)
                acc = chain16r<SAR>(sD, R8, acc, w[q], K8);
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

static_assert(kSegBytes % 4096 == 0 && kSegBytes % 64 == 0, "segments are whole 4 KiB blocks and 64 lane spans");

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

}  // namespace fdfs
