// Run-parallel CRC32_ex building blocks (device side) of crc_seg_kernel
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


// ---- the table fold (crc_tab_kernel: files below kFoldMinBytes) ---------
// Zero-init CRC state of the (masked) bytes [Ap, Ap+len) of one segment,
// computed by the whole wave.  Vectors are 16-byte aligned in memory and the
// 4 KiB block grid is aligned to the segment's last full vector, so the only
// partial vector is the first (leading neutral bytes do not change a
// zero-init state).  See DESIGN.md "K2 segmented CRC" for the algebra.
// The tables are the rotated, replicated slice-by-8 form (64 KiB,
// conflict-free; fdfs_device.hpp chain16r) of Dc for the signed variant (its
// data is folded raw: Dc absorbs the complement) and of D for the unsigned
// one, with K = K8.
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

// ---- the sparse fold (fdfs_tables.hpp fold_exp) -----------
// A wave reduces a run of 16-byte vectors x_0..x_{n-1} (the run's bytes in
// the CRC's domain: complemented for the signed variant, the file's first 4
// bytes XOR 0xFF for the unsigned one, bytes before the run's start 0) to its
// last D = e_4 vectors: c_j = x_j ^ sum_{k<4} c_{j - d_k}, d_k = D - e_k,
// where only positions j <= n - 1 - D pass their value on.  The crc0 of c's
// last D vectors (the slice-by-16 fold in 4 KiB blocks, zeros in front) is
// the run's crc0.  Per vector: one LDS-DMA load, five ds_read_b128 and one
// ds_write_b128 on a per-wave ring, 8 XOR-type ops -- against 16 table
// lookups and ~34 VALU for the slice-by-8 fold of the same 16 bytes.
constexpr int kFoldTaps = kFoldTerms - 1;
constexpr int kFoldRing = 1024;                     // ring positions (c_j at slot j & 1023)
constexpr int kFoldPhases = kFoldRing / 64;         // steps until a slot comes round again
constexpr int kFoldSlots = kFoldRing + 64;          // + a mirror of slots 0..63 (reads never wrap)
constexpr int kFoldAhead = 4;                       // 1 KiB steps in flight per wave
constexpr int kFoldRingBytes = kFoldSlots * 16;
__host__ __device__ constexpr int fold_d(bool sar) { return fold_exp(sar, kFoldTerms - 1); }
static_assert(fold_d(true) - fold_exp(true, kFoldTerms - 2) >= 64 &&
                  fold_d(false) - fold_exp(false, kFoldTerms - 2) >= 64,
              "a step's 64 vectors do not feed each other");
static_assert(64 * kFoldAhead + 63 + fold_d(true) < kFoldRing && 64 * kFoldAhead + 63 + fold_d(false) < kFoldRing,
              "a slot is refilled only after its value's last use");
static_assert(kFoldTaps == 4, "fold5 takes four taps");

// LDS byte address of a __shared__ object.
__device__ __forceinline__ uint32_t lds_addr(const void *p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

// One 1 KiB step of the run (vectors blk[0..63], lane j -> blk[j] at byte
// offset loff = 16 j) into the ring slots at LDS address `slot`: one
// non-temporal LDS-DMA instruction.  Inline asm: with the builtin, hipcc
// waits for every outstanding LDS-DMA load before any LDS read, which would
// leave one step in flight; here the waits are counted (fold_wait).  The
// slots it fills last held positions kFoldRing - 64 kFoldAhead back, whose
// last reads were consumed by the XORs of earlier steps (program order), so
// no LDS wait is needed before it.  M0 is an operand hipcc writes; one wait
// state between that write and the DMA.
__device__ __forceinline__ void fold_issue(const uint4 *blk, uint32_t slot, uint32_t loff)
{
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 offset:0 nt" : : "v"(loff), "s"(blk), "{m0}"(slot) : "memory");
}

// Until at most k steps issued after the one about to be folded are in
// flight (vector memory operations complete in issue order).
__device__ __forceinline__ void fold_wait(int k)
{
    switch (k) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    }
}
static_assert(kFoldAhead == 4, "fold_wait covers 0..4");

// c = x ^ s0 ^ s1 ^ s2 ^ s3 per dword, x complemented first for the signed
// variant: two v_bitop3 per dword.
template <bool SAR>
__device__ __forceinline__ uint32_t fold5(uint32_t x, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3)
{
    const uint32_t t = __builtin_amdgcn_bitop3_b32(s0, s1, s2, 0x96);
    return __builtin_amdgcn_bitop3_b32(x, t, s3, SAR ? 0x69 : 0x96);  // 0x69 = ~(a ^ b ^ c)
}

// A run's fold state and steps (one wave; ring = this wave's kFoldSlots
// vectors, generic pointer and LDS address).
template <bool SAR>
struct FoldRun {
    static constexpr int D = fold_d(SAR);
    const uint4 *v;  // the run's vector grid (16-byte aligned)
    uint4 *ring;
    uint32_t ring_lds, loff;
    int64_t n, nsteps, lim;  // vectors, 64-vector steps, last position that passes its value on
    int64_t a0;
    bool xor4;
    int lane;

    __device__ void issue(int64_t st) const  // step st's DMA (st < nsteps)
    {
        const uint32_t slot = ring_lds + 16u * (uint32_t)((64 * st) & (kFoldRing - 1));
        if (64 * st + 64 <= n) {
            fold_issue(v + 64 * st, slot, loff);
        } else {  // the last, partial step: lanes past the end load the run's last vector
            const int64_t last = n - 1 - 64 * st;
            fold_issue(v + 64 * st, slot, 16u * (uint32_t)(lane < last ? lane : last));
        }
    }

    // Fold step st (st % kFoldPhases == PH: every ring offset is a
    // constant).  FAST: a step of the run's body -- step st + kFoldAhead is
    // whole and issued here, kFoldAhead steps are in flight after this one,
    // all 64 positions are inside the run and all their sources pass on -- so
    // no bounds, masks or branches.  The others (the first kFoldPhases steps
    // and the last few) check.
    template <int PH, bool FAST>
    __device__ void step(int64_t st) const
    {
        constexpr int base = 64 * PH;
        if constexpr (FAST) {
            fold_issue(v + 64 * (st + kFoldAhead),
                       ring_lds + 16u * (uint32_t)((base + 64 * kFoldAhead) & (kFoldRing - 1)), loff);
            fold_wait(kFoldAhead);
        } else {
            if (st + kFoldAhead < nsteps)
                issue(st + kFoldAhead);
            const int64_t after = nsteps - 1 - st;
            fold_wait(after < kFoldAhead ? (int)after : kFoldAhead);
        }
        const uint4 *rl = ring + lane;
        uint4 x = rl[base];
        uint4 sv[kFoldTaps];
#pragma unroll
        for (int k = 0; k < kFoldTaps; k++)
            sv[k] = rl[(base - (D - fold_exp(SAR, k)) + kFoldRing) & (kFoldRing - 1)];
        const int64_t j = 64 * st + lane;
        if constexpr (!FAST) {
            if (st == 0 && lane < 2)
                x = seg_fix_vector<SAR>(x, 16 * j, a0, xor4);  // the partial first vector; the first 4 file bytes
            constexpr int dmin = D - fold_exp(SAR, kFoldTaps - 1);
            if (64 * st + 63 - dmin > lim) {  // the run's last steps: positions past lim do not pass on
#pragma unroll
                for (int k = 0; k < kFoldTaps; k++)
                    if (j - (D - fold_exp(SAR, k)) > lim)
                        sv[k] = make_uint4(0, 0, 0, 0);
            }
        }
        uint4 c;
        c.x = fold5<SAR>(x.x, sv[0].x, sv[1].x, sv[2].x, sv[3].x);
        c.y = fold5<SAR>(x.y, sv[0].y, sv[1].y, sv[2].y, sv[3].y);
        c.z = fold5<SAR>(x.z, sv[0].z, sv[1].z, sv[2].z, sv[3].z);
        c.w = fold5<SAR>(x.w, sv[0].w, sv[1].w, sv[2].w, sv[3].w);
        if (FAST || j < n) {
            uint4 *wl = ring + lane;
            wl[base] = c;
            if constexpr (PH == 0)
                wl[kFoldRing] = c;  // the mirror of slots 0..63
        }
    }

    template <int PH, bool FAST>
    __device__ void steps_from(int64_t g) const  // steps g + PH .. g + kFoldPhases - 1
    {
        if constexpr (PH < kFoldPhases) {
            if (!FAST && g + PH >= nsteps)
                return;
            step<PH, FAST>(g + PH);
            steps_from<PH + 1, FAST>(g);
        }
    }
};

// Zero-init CRC state (crc0) of the bytes [Ap, Ap + len) of one run of a
// file (first: the run starts at the file's first byte), computed by the
// whole wave.  Vectors are 16-byte aligned in memory; the first is partial
// (bytes before Ap neutral), the <= 15 bytes after the last full vector are
// folded byte-wise.  sD: the plain slice-by-16 tables (the signed variant's
// data is complemented before the fold), sA: ADV4032, sT: the byte table.
template <bool SAR>
__device__ __forceinline__ uint32_t crc_run(const uint32_t *sD, const uint32_t *sA, const uint32_t *sT,
                                            const uint32_t *sR, uint32_t K16, const uint8_t *Ap, uint64_t len,
                                            bool first, uint4 *ring, uint32_t ring_lds, int lane)
{
    FoldRun<SAR> F;
    F.a0 = (int64_t)((uintptr_t)Ap & 15u);
    F.v = reinterpret_cast<const uint4 *>(Ap - F.a0);
    const int64_t e_off = F.a0 + (int64_t)len;
    F.n = e_off >> 4;
    F.xor4 = !SAR && first;
    F.ring = ring;
    F.ring_lds = ring_lds;
    F.lane = lane;
    F.loff = 16u * (uint32_t)lane;
    uint32_t state = 0;
    if (F.n > 0) {
        constexpr int D = FoldRun<SAR>::D;
        F.nsteps = (F.n + 63) >> 6;
        F.lim = F.n - 1 - D;
        // positions -D..-1 read as zero (slots kFoldRing - D .. kFoldRing - 1;
        // the first kFoldAhead steps' DMA fills slots 0 .. 64 kFoldAhead - 1)
        constexpr int z0 = (kFoldRing - D) & ~63;
        static_assert(z0 >= 64 * kFoldAhead, "zeroed slots apart from the first DMA");
#pragma unroll
        for (int m = z0; m < kFoldRing; m += 64)
            ring[m + lane] = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int st = 0; st < kFoldAhead; st++)
            if (st < F.nsteps)
                F.issue(st);
        // fast steps: st + kFoldAhead whole (64 (st + kFoldAhead + 1) <= n)
        // and every source passing on (64 st + 63 - dmin <= lim)
        constexpr int dmin = D - fold_exp(SAR, kFoldTaps - 1);
        int64_t nfast = (F.n >> 6) - kFoldAhead;
        if (F.lim + dmin - 63 < 0)
            nfast = 0;
        else if (((F.lim + dmin - 63) >> 6) + 1 < nfast)
            nfast = ((F.lim + dmin - 63) >> 6) + 1;
        for (int64_t g = 0; g < F.nsteps; g += kFoldPhases) {
            if (g > 0 && g + kFoldPhases <= nfast)
                F.template steps_from<0, true>(g);
            else
                F.template steps_from<0, false>(g);
        }
        // the remainder, c's last min(D, n) vectors, in 4 KiB blocks aligned
        // to its end (zeros in front): lane l folds block vectors 4 l .. 4 l + 3
        const int64_t first_rem = F.n - D > 0 ? F.n - D : 0;
        const int64_t J = (F.n - first_rem + 255) >> 8;
        uint32_t acc = 0;
        for (int64_t jb = 0; jb < J; jb++) {
            if (jb > 0)
                acc = apply4(sA, acc);  // advance 4032 B to this lane's next piece
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int64_t p = F.n - 256 * (J - jb) + 4 * lane + q;
                uint4 w = make_uint4(0, 0, 0, 0);
                if (p >= first_rem)
                    w = ring[p & (kFoldRing - 1)];
                acc = chain16<SAR>(sD, acc, w, K16);
            }
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
    const int64_t t0 = (16 * F.n > F.a0) ? 16 * F.n : F.a0;
    for (int64_t o = t0; o < e_off; o++) {
        uint32_t b = Ap[o - F.a0];
        if (SAR || (F.xor4 && o < F.a0 + 4))
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
