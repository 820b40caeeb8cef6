// sig_hash_kernel: CRC32 + CALC_HASH_CODES4 (FDFS_SIG_HASH, config 2).
//
// One LANE per file (ELFHash is a byte-serial recurrence), 64 files of
// near-equal size per wave (size-binned order), each lane streaming its own
// file in whole 128-byte lines (8 x 16-byte loads per step, line-aligned
// window: one L1/L2 line per lane per step).
//
// The kernel is VALU-issue bound.  On gfx950 v_lshl_add / v_bfe / v_perm /
// v_dot4 / v_mul_lo / SDWA issue at half rate (profiles/r01/
// ubench_valu_rate2.txt), so the per-byte cost is counted in full-rate slots
// and each hash is placed where it is cheapest:
//
//  * CRC32_ex: the lane fold over whole 128-byte steps (fdfs_device.hpp
//    lane_fold_dw: a 32-register ring, 6-7 v_bitop3 per dword, no table
//    lookups); slice-by-16 tables in LDS only for the lane-serial
//    head and tail bytes and the fold's final 128 bytes.
//  * ELFHash_ex: 4 VALU per byte (shift, SDWA byte add, shift, bitop3),
//    one asm statement per word (fdfs_device.hpp elf_word4).
//  * simple_hash_ex / Time33Hash_ex: over a 128-byte step each hash is
//    h' = M^128 h + sum_pos M^(127-pos) b_pos (mod 2^32), i.e. a dot product
//    of the bytes with fixed coefficients -- a contraction, so it runs on the
//    i8 matrix cores.  The coefficients are split into 4 balanced int8 digit
//    planes; per 16-byte vector one v_mfma_i32_16x16x64_i8 per hash takes
//    the 64 lanes' vectors as A (lane l's 16 bytes are row l & 15 of k-block
//    l >> 4) and a block-diagonal B (fdfs_tables.cpp), giving the 4 planes
//    of every file's dot.  The running hash lives in the accumulator layout
//    as 4 planes per file: once per group of 8 steps the planes are
//    multiplied by M^1024 (and the 128 * sum(digits) bias of the
//    b ^ 0x80 = b - 128 encoding is added), which is Horner's rule on each
//    plane (multiplying by M is linear mod 2^32); B carries the group's
//    1024 coefficients.  At the end the planes are summed (sum P_j << 8j),
//    moved back to the file's lane, and the zero-padded steps of files
//    shorter than the wave's longest are undone with M^-128 powers.
//
// Reference loops replaced: storage/storage_dio.c:465-515 (CRC32_ex and
// CALC_HASH_CODES4 per chunk, FINISH_HASH_CODES4), storage/storage_service.c:
// 106-120 (STORAGE_GEN_FILE_SIGNATURE).
#include "fdfs_device.hpp"
#include "fdfs_kernels.hpp"

namespace fdfs {

// 256 threads: four workgroups (18 KB of tables each) per CU at 4 waves per
// SIMD; 512-thread workgroups ran 4 % slower (profiles/r01/hash_block_ab.txt).
constexpr int kHashBlock = 256;

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// All four CALC_HASH_CODES4 hashes of one 16-byte vector on the lane.
template <bool SAR>
__device__ __forceinline__ void h4_lane(const uint32_t *sD, uint32_t K16, uint4 q, bool small, uint32_t &c,
                                        uint32_t &e, uint32_t &s, uint32_t &t)
{
    if (small)
        c = chain16<SAR>(sD, c, q, K16);
    elf_word4<SAR, false>(q.x, e);
    elf_word4<SAR, false>(q.y, e);
    elf_word4<SAR, false>(q.z, e);
    elf_word4<SAR, true>(q.w, e);
    s = poly_word<31>(s, q.x);
    t = poly_word<33>(t, q.x);
    s = poly_word<31>(s, q.y);
    t = poly_word<33>(t, q.y);
    s = poly_word<31>(s, q.z);
    t = poly_word<33>(t, q.z);
    s = poly_word<31>(s, q.w);
    t = poly_word<33>(t, q.w);
}

// (a & m) ^ 0x80808080 in one VALU op (v_bitop3_b32, truth table 0x6A):
// the b - 128 int8 operand of a lane, zero data past the file's end.  A
// builtin, not an asm statement: its result feeds the MFMA's A operand
// directly, and only an instruction hipcc can see gets the VALU-write ->
// MFMA-read wait states padded (round 2's asm form left one state where two
// are required; tests/test_isa.py checks the shipped code object).
__device__ __forceinline__ uint32_t and_xor80(uint32_t a, uint32_t m)
{
    return __builtin_amdgcn_bitop3_b32(a, m, 0x80808080u, 0x6a);
}

// ELFHash_ex of one big file on a workgroup of its own (one-shot batches of
// at most lat_files files with at most chain_cap big files; sig_hash_kernel's
// first workgroups).  A lane alone on its SIMD issues about one instruction
// per 4 cycles, so the chain lane's own byte extraction and loads are time on
// the chain: here wave 1 puts the file's bytes one per dword into an LDS ring
// (two slots of 2 KiB of file, 32 coalesced byte loads per lane per slot) and
// wave 0 runs the three dependent VALU per byte alone (v_lshl_add_u32 with
// the byte, shift, v_bitop3), reading each 64 bytes' dwords one group ahead.
// CRC, simple_hash and Time33 of a big file come from the segmented kernels
// (big_patch_kernel); this writes the signature's size and ELF fields and
// codes[1].  Waves 2 and 3 only keep the barrier count.
constexpr uint32_t kElfSlot = 2048;  // file bytes per LDS slot (8 KiB of byte-dwords)

template <bool SAR>
__device__ __forceinline__ void elf_byte(uint32_t b, uint32_t &e, uint32_t &y)
{
    const uint32_t t = (e << 4) + b;
    y = SAR ? (uint32_t)((int32_t)t >> 24) : (t >> 24);
    e = t ^ (y & 0xFFFFFFF0u);  // dirty top nibble (elf_exact_after)
}

template <bool SAR>
__device__ __forceinline__ void elf_chain_wg(const uint8_t *p, uint64_t L, uint32_t f, uint32_t *ring,
                                             uint8_t *sig_out, int32_t *codes_out, fdfs_gpu_file_state *fs)
{
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint64_t nslots = uniform64((L + kElfSlot - 1) / kElfSlot);
    if (wv == 1) {
        auto fill = [&](uint32_t *slot, uint64_t s) {
            const uint8_t *q = p + s * kElfSlot;
            const uint64_t nb = L - s * kElfSlot;  // > 0
#pragma unroll
            for (int j0 = 0; j0 < (int)(kElfSlot / 64); j0 += 16) {
                uint32_t v[16];
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const uint32_t k = (j0 + u) * 64 + lane;
                    v[u] = k < nb ? q[k] : 0u;
                }
#pragma unroll
                for (int u = 0; u < 16; u++)
                    slot[(j0 + u) * 64 + lane] = v[u];
            }
        };
        if (nslots)
            fill(ring, 0);
        __syncthreads();
        for (uint64_t s = 0; s < nslots; s++) {
            if (s + 1 < nslots)
                fill(ring + ((s + 1) & 1) * kElfSlot, s + 1);
            __syncthreads();
        }
        return;
    }
    if (wv != 0) {
        __syncthreads();
        for (uint64_t s = 0; s < nslots; s++)
            __syncthreads();
        return;
    }
    __builtin_amdgcn_s_setprio(3);
    // the same chain on every lane: an opaque per-lane zero keeps it in VGPRs
    // (hipcc would run a wave-uniform chain on the scalar unit, with a
    // v_readfirstlane per step)
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    // INIT_HASH_CODES4's 0, or the chunk's state (fdfs_gpu_update_batch);
    // y < 0: exact as it stands
    uint32_t e = z ^ (fs ? (uint32_t)fs->hash_codes[1] : 0u), y = 0x80000000u;
    __syncthreads();
    for (uint64_t s = 0; s < nslots; s++) {
        const uint4 *R = reinterpret_cast<const uint4 *>(ring + (s & 1) * kElfSlot);
        const uint64_t rem = L - s * kElfSlot;
        const uint32_t nb = (uint32_t)uniform64(rem < kElfSlot ? rem : kElfSlot);
        const uint32_t ng = nb >> 6;  // whole 64-byte groups
        // group g's steps from cur while a quarter of group g + 1's reads
        // goes out before each quarter's steps (at most 8 LDS reads
        // outstanding: lgkmcnt counts to 15); two buffers in turn, no copies
        auto group = [&](const uint4 (&cur)[16], uint4 (&nxt)[16], const uint4 *N) {
#pragma unroll
            for (int h = 0; h < 4; h++) {
#pragma unroll
                for (int k = 4 * h; k < 4 * h + 4; k++)
                    nxt[k] = N[k];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 4 * h; k < 4 * h + 4; k++) {
                    elf_byte<SAR>(cur[k].x, e, y);
                    elf_byte<SAR>(cur[k].y, e, y);
                    elf_byte<SAR>(cur[k].z, e, y);
                    elf_byte<SAR>(cur[k].w, e, y);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        uint4 A[16], B[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
            A[k] = R[k];
        uint32_t g = 0;
        for (; g + 2 <= ng; g += 2) {
            group(A, B, R + 16 * (g + 1));
            group(B, A, R + 16 * (g + 2 < ng ? g + 2 : 0));
        }
        if (g < ng)  // an odd group count: the last group (the reads go to B unused)
            group(A, B, R);
        const uint32_t *Rw = reinterpret_cast<const uint32_t *>(R);
        for (uint32_t k = ng << 6; k < nb; k++)  // the slot's last < 64 bytes (the file's end)
            elf_byte<SAR>(Rw[k], e, y);
        __syncthreads();
    }
    e = elf_exact_after(e, y);
    if (fs) {  // the state-carrying update: ELF and the byte count (the CRC and
               // polynomials come from big_patch_state_kernel)
        if (lane == 0) {
            fs->hash_codes[1] = (int32_t)e;
            uint32_t cnt[2] = {fs->md5_count[0], fs->md5_count[1]};
            count_add(cnt, L);
            fs->md5_count[0] = cnt[0];
            fs->md5_count[1] = cnt[1];
        }
        return;
    }
    if (lane == 0) {
        if (sig_out) {  // be64 size at 0, be32 ELF at 12 (big_patch_kernel writes the CRC, simple, Time33)
            uint32_t *sp = reinterpret_cast<uint32_t *>(sig_out + 24ull * f);
            sp[0] = bswap32((uint32_t)(L >> 32));
            sp[1] = bswap32((uint32_t)L);
            sp[3] = bswap32(e);
        }
        if (codes_out)
            codes_out[4ull * f + 1] = (int32_t)e;
    }
}

// ST (fdfs_gpu_update_batch): the lane continues the chunk's
// StorageFileContext-shaped state (crc32, file_hash_codes) instead of
// INIT_HASH_CODES4 and writes it back unfinalised; every step above is a
// recurrence from whatever state it starts in (the polynomial planes start
// from the lane's running value), so nothing else changes.
// Occupancy: the production instantiations fit four waves per SIMD (128
// registers) with AGPR accumulators as compiled.  Asking for four waves
// explicitly made hipcc move the ST form's accumulators to VGPRs (caught by
// tests/test_isa.py), so none is asked for.
template <bool SAR, bool ST>
__global__ __launch_bounds__(kHashBlock) __attribute__((amdgpu_waves_per_eu(1))) void sig_hash_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint64_t *__restrict__ sizes, const uint32_t *__restrict__ order, uint32_t n,
    const DevTables *__restrict__ tabs, const uint64_t *__restrict__ big_min_p,
    uint32_t *__restrict__ crc_out, uint8_t *__restrict__ sig_out, int32_t *__restrict__ codes_out,
    fdfs_gpu_file_state *__restrict__ states, const uint32_t *__restrict__ sidx,
    const uint32_t *__restrict__ nbig_p, uint32_t chain_slots)
{
    __shared__ __attribute__((aligned(16))) uint32_t sD[16 * 256];  // also elf_chain_wg's ring
    __shared__ uint32_t sT[256];
    constexpr int SV = 8;             // vectors per step: one 128-byte line
    constexpr int NSETS = 2;          // register sets of loads in flight
    constexpr uint32_t SB = 16 * SV;  // bytes per step
    // 128-byte steps per Horner multiply of the accumulators (the B operands
    // carry the coefficients of the whole group: fdfs_tables.hpp BG)
    constexpr int HG = kHornerGroup;
    // The MFMA B operands, compacted: lane l's 16 bytes for (hash h, vector
    // q) are digit plane l & 3 of that vector's coefficients when l lies on
    // the block diagonal ((l >> 4) == ((l & 15) >> 2), fdfs_tables.cpp) and
    // zero otherwise -- five distinct 16-byte rows per (h, q): 1.25 KB of
    // LDS per step instead of 16 KB (rows 0-3 = lanes 0-3's B, row 4 = zero),
    // for the HG steps of a Horner group.
    __shared__ uint4 sB[2 * SV * HG * 5];
    lds_fill(sD, &tabs->t.D[0][0], 16 * 256);
    lds_fill(sT, tabs->t.T, 256);
    for (int i = threadIdx.x; i < 2 * SV * HG * 5; i += blockDim.x) {
        const int h = i / (SV * HG * 5), q = (i / 5) % (SV * HG), r = i % 5;
        const int8_t *row = &tabs->pm.BG[h][q][r & 3][0];
        sB[i] = r < 4 ? *reinterpret_cast<const uint4 *>(row) : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    const int brow = ((threadIdx.x & 63) >> 4) == ((threadIdx.x & 15) >> 2) ? (threadIdx.x & 3) : 4;

    // The first chain_slots workgroups: big file i < *nbig (when *nbig <=
    // chain_slots) on workgroup i (elf_chain_wg); the lanes skip those files.
    uint32_t nchain = 0;
    if (chain_slots) {
        const uint32_t nb = __builtin_amdgcn_readfirstlane(*nbig_p);
        nchain = nb <= chain_slots ? nb : 0;
        if (blockIdx.x < chain_slots) {
            if (blockIdx.x < nchain) {
                const uint32_t fc = order[blockIdx.x];
                if (fc < n)  // else a stale order entry (flagged by big_plan_kernel)
                    elf_chain_wg<SAR>(base + offs[fc], sizes[fc], fc, sD, sig_out, codes_out,
                                      ST ? states + (sidx ? sidx[fc] : fc) : nullptr);
            }
            return;
        }
    }
    const int lane = threadIdx.x & 63;
    const uint32_t wave0 = (blockIdx.x - chain_slots) * blockDim.x + (threadIdx.x & ~63u);
    if (wave0 >= n)  // whole wave past the batch (wave-uniform: MFMAs below need every lane)
        return;
    const uint32_t i = wave0 + lane;
    bool valid = i < n;
    const uint32_t K16 = tabs->t.K16;
    const uint8_t *safe = reinterpret_cast<const uint8_t *>(tabs);  // >= 128 readable bytes
    uint32_t f = valid ? order[i] : 0;
    if (f >= n) {  // a stale order entry (the binning flagged it): no file
        valid = false;
        f = 0;
    }
    if (nchain && valid && sizes[f] >= *big_min_p)  // a chain workgroup's file
        valid = false;
    const uint64_t L = valid ? sizes[f] : 0;
    const uint8_t *p = valid ? base + offs[f] : safe;
    uint32_t c = 0xFFFFFFFFu;  // CRC32_XINIT (storage/storage_service.c:7149)
    uint32_t e = 0, s = 0, t = 0;  // INIT_HASH_CODES4 (storage/storage_service.c:7156)
    fdfs_gpu_file_state *fs = nullptr;
    if constexpr (ST) {
        if (valid) {
            fs = states + (sidx ? sidx[f] : f);
            c = (uint32_t)fs->crc32;
            e = (uint32_t)fs->hash_codes[1];
            s = (uint32_t)fs->hash_codes[2];
            t = (uint32_t)fs->hash_codes[3];
        }
    }
    // Files of >= big_min bytes leave their CRC, simple_hash and Time33 to
    // segment-parallel kernels (launch_sig_lane runs them before this one
    // and patches the outputs after) and keep only ELFHash here: their waves
    // are few and issue-bound, the rest is ~half of their instructions, and
    // once a wave's smaller files have ended its CRC blocks run with an
    // empty exec mask (branched over) and its MFMA steps are skipped.
    const uint64_t big_min = big_min_p ? *big_min_p : ~0ull;  // big_plan_kernel's T
    const bool small = L < big_min;

    // bytes to 16-byte alignment, then vectors to 128-byte alignment (lane-serial)
    uint64_t head = (16u - ((uintptr_t)p & 15u)) & 15u;
    if (head > L)
        head = L;
    for (uint64_t k = 0; k < head; k++) {
        const uint32_t b = p[k];
        if (small)
            c = crc_byte<SAR>(sT, c, b);
        h3_byte<SAR>(b, e, s, t);
    }
    const uint4 *v = reinterpret_cast<const uint4 *>(p + head);
    const uint64_t nvec = (L - head) >> 4;
    uint64_t lead = ((SB - ((uintptr_t)v & (SB - 1))) & (SB - 1)) >> 4;
    if (lead > nvec)
        lead = nvec;
    for (uint64_t j = 0; j < lead; j++)
        h4_lane<SAR>(sD, K16, v[j], small, c, e, s, t);

    // whole steps: the wave steps in lockstep to its longest file
    const uint32_t nsteps = (uint32_t)((nvec - lead) / SV);
    uint32_t nmax = nsteps;
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        const uint32_t y = __shfl_xor(nmax, o);
        nmax = y > nmax ? y : nmax;
    }
    if (nmax) {
        const uint32_t m31 = tabs->pm.m1024[0];
        const uint32_t m33 = tabs->pm.m1024[1];
        const int col = lane & 15, j = col & 3, g = col >> 2;
        const int32_t kk31 = tabs->pm.KG[0][j];
        const int32_t kk33 = tabs->pm.KG[1][j];
        const i32x4 k31 = {kk31, kk31, kk31, kk31};
        const i32x4 k33 = {kk33, kk33, kk33, kk33};
        // accumulator element r of this lane: plane j of the file in lane
        // 16 g + 4 (lane >> 4) + r; plane 0 starts from the lane-serial state
        i32x4 C31, C33;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int src = 16 * g + 4 * (lane >> 4) + r;
            const uint32_t s0 = __shfl(s, src), t0 = __shfl(t, src);
            C31[r] = j == 0 ? (int)s0 : 0;
            C33[r] = j == 0 ? (int)t0 : 0;
        }
        const uint4 *w = v + lead;
        // The CRC of the steps: the lane fold in 32 registers, the CRC state
        // so far entering as the first step's first dword (fdfs_tables.hpp Y4)
        uint32_t ring[32];
#pragma unroll
        for (int k = 0; k < 32; k++)
            ring[k] = 0;
        uint32_t zin = c ^ ((SAR && (int32_t)c < 0) ? tabs->t.Y4 : 0u);
        // One 128-byte step: lane hashes for files not yet ended, then the
        // two polynomial MFMAs per vector for every lane.
        // Steps only run the polynomial MFMAs while a lane below big_min is
        // still hashing (big files get simple/Time33 from poly_seg_kernel):
        // nexec counts them for the padding undo below.
        uint32_t nexec = 0;
        // steps of the last Horner group that ran their MFMAs (< HG: the
        // group's bias for the steps after them is taken back at the end)
        uint32_t egrp = HG;
        // the last ELF step's t >> 24 (negative: e is exact as it stands)
        uint32_t ylast = 0x80000000u;
        // The step's pieces arrive interleaved over lane pairs (issue_p
        // below) and are transposed back to their files' lanes: one
        // transpose stage per quarter line, just before its two vectors are
        // hashed.
        auto ptr = [](u32x4 (&a)[SV], int p) {
            uint32_t r0[4], r1[4], t[4];
#pragma unroll
            for (int d = 0; d < 4; d++) {
                r0[d] = a[2 * p][d];
                r1[d] = a[2 * p + 1][d];
            }
            pair_transpose(r0, r1, t);
#pragma unroll
            for (int d = 0; d < 4; d++) {
                a[2 * p][d] = r0[d];
                a[2 * p + 1][d] = t[d];
            }
        };
        auto step = [&](u32x4 (&a)[SV], bool ok, uint32_t stp) {
            const bool mon = __any(ok && small);
            // position of the step in its Horner group (wave-uniform); the
            // group's first step scales the planes by M^(128 HG) and adds the
            // group's bias, and counts the group's HG steps for the undo
            const uint32_t sg = stp & (HG - 1);
            if (mon) {
                nexec += sg == 0 ? (uint32_t)HG : 0u;
                egrp = sg + 1;
            }
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if (!mon || sg != 0)
                    break;
                C31[r] = (int)((uint32_t)C31[r] * m31) + k31[r];
                C33[r] = (int)((uint32_t)C33[r] * m33) + k33[r];
            }
#pragma unroll
            for (int q = 0; q < SV; q++) {
                if ((q & 1) == 0) {
                    __builtin_amdgcn_sched_barrier(0);
                    ptr(a, q >> 1);
                    __builtin_amdgcn_sched_barrier(0);
                }
                const uint4 aq = make_uint4(a[q][0], a[q][1], a[q][2], a[q][3]);
                if (ok) {
                    if (small) {
                        ring[4 * q + 0] = lane_fold_dw<SAR>(ring, 4 * q + 0, q == 0 ? aq.x ^ zin : aq.x);
                        ring[4 * q + 1] = lane_fold_dw<SAR>(ring, 4 * q + 1, aq.y);
                        ring[4 * q + 2] = lane_fold_dw<SAR>(ring, 4 * q + 2, aq.z);
                        ring[4 * q + 3] = lane_fold_dw<SAR>(ring, 4 * q + 3, aq.w);
                    }
                    // the top nibble stays dirty across vectors (each step
                    // shifts it out); made exact once after the steps from
                    // the last t's sign (elf_exact_after)
                    elf_vec16y<SAR>(aq, e, ylast);
                }
                if (!mon)
                    continue;
                // b - 128 as int8 (b ^ 0x80); a padded step is all-zero data
                const uint32_t msk = ok ? 0xFFFFFFFFu : 0u;
                const i32x4 A = {(int)and_xor80(aq.x, msk), (int)and_xor80(aq.y, msk),
                                 (int)and_xor80(aq.z, msk), (int)and_xor80(aq.w, msk)};
                // the step's vector q carries coefficients M^(SB-1-pos) (B's vector q)
                const uint4 b31 = sB[(0 * SV * HG + sg * SV + q) * 5 + brow];
                const uint4 b33 = sB[(1 * SV * HG + sg * SV + q) * 5 + brow];
                const i32x4 B31 = {(int)b31.x, (int)b31.y, (int)b31.z, (int)b31.w};
                const i32x4 B33 = {(int)b33.x, (int)b33.y, (int)b33.z, (int)b33.w};
                C31 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B31, C31, 0, 0, 0);
                C33 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B33, C33, 0, 0, 0);
            }
            zin = 0;  // taken by every lane's first step (all lanes start at step 0)
        };
        // The next step's line is loaded while this one is hashed: two
        // register sets, asm loads (hipcc would sink plain loads to their
        // use), issued unconditionally (past-the-end steps read `safe`) so no
        // register an asm load is still writing is ever copied.
        u32x4 RS[NSETS][SV];
        auto issue = [&](u32x4 (&R)[SV], uint32_t stp) {
            const uint8_t *ln = stp < nsteps ? reinterpret_cast<const uint8_t *>(w + SV * (uint64_t)stp) : safe;
#pragma unroll
            for (int q = 0; q < SV; q++)
                asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(R[q]) : "v"(ln), "i"(16 * q) : "memory");
        };
        // Pair-cooperative loads (round 4): lane j of pair P loads piece
        // 2p + j of pair-file k's line into R[2p + k]: 32 contiguous bytes
        // per lane pair per instruction, one transpose stage (4 VALU per
        // vector instead of the rounds-2-3 quad form's 8): 8.41 against
        // 8.58-8.60 ms (profiles/r04/pair_loads_ab.txt).  The pair's line
        // addresses are broadcast by DPP quad_perm [k,k,2+k,2+k].
        auto issue_p = [&](u32x4 (&R)[SV], uint32_t stp) {
            const uint8_t *ln = stp < nsteps ? reinterpret_cast<const uint8_t *>(w + SV * (uint64_t)stp) : safe;
            const uint64_t a = reinterpret_cast<uint64_t>(ln);
            const uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
            auto ld = [&](int k, uint32_t lk, uint32_t hk) {
                const uint8_t *pk = reinterpret_cast<const uint8_t *>(((uint64_t)hk << 32 | lk) + 16u * (lane & 1));
                asm volatile("global_load_dwordx4 %0, %1, off offset:0" : "=v"(R[k]) : "v"(pk) : "memory");
                asm volatile("global_load_dwordx4 %0, %1, off offset:32" : "=v"(R[2 + k]) : "v"(pk) : "memory");
                asm volatile("global_load_dwordx4 %0, %1, off offset:64" : "=v"(R[4 + k]) : "v"(pk) : "memory");
                asm volatile("global_load_dwordx4 %0, %1, off offset:96" : "=v"(R[6 + k]) : "v"(pk) : "memory");
            };
#define PBC(S) (uint32_t) __builtin_amdgcn_mov_dpp((int)lo, S, 0xF, 0xF, false), \
               (uint32_t) __builtin_amdgcn_mov_dpp((int)hi, S, 0xF, 0xF, false)
            ld(0, PBC(0xA0));
            ld(1, PBC(0xF5));
#undef PBC
        };
        // R is the oldest of the NSETS sets in flight
        auto wait_older = [&](u32x4 (&R)[SV]) {
            static_assert(NSETS == 2 && SV == 8, "128-byte steps: two sets of 8 registers");
            asm volatile("s_waitcnt vmcnt(8)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]) :: "memory");
            asm volatile("" : "+v"(R[4]), "+v"(R[5]), "+v"(R[6]), "+v"(R[7]));
        };
        auto drain = [&]() {
#pragma unroll
            for (int k = 0; k < NSETS; k++)
                asm volatile("s_waitcnt vmcnt(0)"
                             : "+v"(RS[k][0]), "+v"(RS[k][1]), "+v"(RS[k][2]), "+v"(RS[k][3]), "+v"(RS[k][4]),
                               "+v"(RS[k][5]), "+v"(RS[k][6]), "+v"(RS[k][7]) :: "memory");
        };
        // Steps [first, end) with NSETS - 1 steps' loads ahead of the one
        // hashed (past-the-end steps load `safe`).
        auto pipeline = [&](auto &&iss_fn, auto &&step_fn, uint32_t first, uint32_t end) {
#pragma unroll
            for (int k = 0; k < NSETS - 1; k++)
                iss_fn(RS[k], first + k);
            for (uint32_t st = first; st < end; st += NSETS) {
#pragma unroll
                for (int k = 0; k < NSETS; k++) {
                    iss_fn(RS[(k + NSETS - 1) % NSETS], st + k + NSETS - 1);
                    wait_older(RS[k]);
                    if (k == 0 || st + k < end)
                        step_fn(RS[k], st + k < nsteps, st + k);
                }
            }
            drain();
        };
        // Small lanes only ever end, so the steps where a lane below big_min
        // is still hashing are a prefix [0, nfull) of the wave's steps.  The
        // rest (waves of big files) hash ELF alone and are bound by its
        // dependent chain: the 3-op form (elf_word4_chain) there.
        uint32_t nfull = small ? nsteps : 0;
#pragma unroll
        for (int o = 32; o; o >>= 1) {
            const uint32_t y = __shfl_xor(nfull, o);
            nfull = y > nfull ? y : nfull;
        }
        if (nfull)
            pipeline(issue_p, step, 0u, nfull);
        // The rest of the steps (waves of big files: ELF alone, its
        // dependent chain the bound).  Four 64-byte load sets here (192 B of
        // lookahead in the same registers) measured 906-962 against 826-940
        // ms on config 1, within that config's run-to-run spread
        // (profiles/r03/hash_pipeline_ab.txt): not kept.
        auto step_chain = [&](u32x4 (&a)[SV], bool ok, uint32_t) {
            if (!ok)
                return;
#pragma unroll
            for (int q = 0; q < SV; q++) {
                elf_word4_chain<SAR, false>(a[q][0], e);
                elf_word4_chain<SAR, false>(a[q][1], e);
                elf_word4_chain<SAR, false>(a[q][2], e);
                elf_word4_chain_y<SAR>(a[q][3], e, ylast);
            }
        };
        if (nfull < nmax)
            pipeline(issue, step_chain, nfull, nmax);
        if (small && nsteps > 0)
            c = lane_fold_finish<SAR>(sD, K16, ring);
        e = elf_exact_after(e, ylast);
        if (nexec && egrp < HG) {  // the last group ran egrp of its HG steps
#pragma unroll
            for (int r = 0; r < 4; r++) {
                C31[r] -= tabs->pm.KGtail[0][egrp][j];
                C33[r] -= tabs->pm.KGtail[1][egrp][j];
            }
        }
        // planes -> value: sum_j P_j << 8j over the lane quad (j = lane & 3),
        // then back to the file's lane; undo the padded steps (M^-SB each)
        uint32_t s31 = 0, s33 = 0;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            uint32_t x = (uint32_t)C31[r] << (8 * j), y = (uint32_t)C33[r] << (8 * j);
            x += __shfl_xor(x, 1);
            y += __shfl_xor(y, 1);
            x += __shfl_xor(x, 2);
            y += __shfl_xor(y, 2);
            // file lane F = 16 g' + 4 h + r has its sum in lane 4 g' + 16 h (g' = F >> 4, h = (F & 15) >> 2)
            const int src = 4 * (lane >> 4) + 16 * ((lane & 15) >> 2);
            const uint32_t xs = __shfl(x, src), ys = __shfl(y, src);
            if ((lane & 3) == r) {
                s31 = xs;
                s33 = ys;
            }
        }
        const uint32_t pad = nexec - nsteps;  // (garbage for big-file lanes: patched)
        s = s31 * pow_dev(tabs->pm.inv128[0], pad);
        t = s33 * pow_dev(tabs->pm.inv128[1], pad);
    }

    for (uint64_t jv = lead + SV * (uint64_t)nsteps; jv < nvec; jv++)
        h4_lane<SAR>(sD, K16, v[jv], small, c, e, s, t);
    for (uint64_t k = head + (nvec << 4); k < L; k++) {  // the last (L - head) & 15 bytes
        const uint32_t b = p[k];
        if (small)
            c = crc_byte<SAR>(sT, c, b);
        h3_byte<SAR>(b, e, s, t);
    }
    if (!valid)
        return;
    if constexpr (ST) {
        // big chunks: crc32, codes 0/2/3 come from big_patch_kernel, which
        // still needs the chunk's starting values there
        if (small) {
            fs->crc32 = (int32_t)c;
            fs->hash_codes[0] = (int32_t)c;
            fs->hash_codes[2] = (int32_t)s;
            fs->hash_codes[3] = (int32_t)t;
        }
        fs->hash_codes[1] = (int32_t)e;
        uint32_t cnt[2] = {fs->md5_count[0], fs->md5_count[1]};
        count_add(cnt, L);
        fs->md5_count[0] = cnt[0];
        fs->md5_count[1] = cnt[1];
        return;
    }
    c ^= 0xFFFFFFFFu;  // CRC32_FINAL / FINISH_HASH_CODES4 (storage/storage_dio.c:500,508)
    if (small)
        crc_out[f] = c;  // else big_patch_kernel puts the segmented CRC in all three outputs
    if (sig_out) {  // STORAGE_GEN_FILE_SIGNATURE (storage/storage_service.c:106-120)
        uint2 *sp = reinterpret_cast<uint2 *>(sig_out + 24ull * f);
        sp[0] = make_uint2(bswap32((uint32_t)(L >> 32)), bswap32((uint32_t)L));
        sp[1] = make_uint2(bswap32(c), bswap32(e));
        sp[2] = make_uint2(bswap32(s), bswap32(t));
    }
    if (codes_out)
        reinterpret_cast<int4 *>(codes_out)[f] = make_int4((int)c, (int)e, (int)s, (int)t);
}

// crc_lane_kernel: CRC32 only (FDFS_SIG_CRC_ONLY) for large batches of small
// files, one lane per file in the size-binned order, the same 128-byte steps
// and pair-cooperative loads as sig_hash_kernel and the lane fold for the
// CRC (fdfs_device.hpp): ~29 VALU per 16 bytes, no table lookups, so the
// loads bound it.  Files >= *big_min_p (kFoldMinBytes for CRC_ONLY,
// big_plan_kernel) take crc_seg_kernel's sparse fold and are skipped here.
// fdfs_gpu_sig_batch routes CRC-only batches of more than 3 lat_files files
// here; smaller ones keep crc_tab_kernel's wave per file (latency).
// Reference loop replaced: storage/storage_dio.c:465-467 (CRC32_ex per
// chunk), storage/storage_dio.c:500 (CRC32_FINAL).
template <bool SAR>
// 137 VGPRs: three waves per SIMD.  Forcing four makes hipcc spill, and a
// spill or copy of a load register an asm load is still writing reads it
// early (measured: half the CRCs wrong), so none is asked for.
__global__ __launch_bounds__(kHashBlock) void crc_lane_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint64_t *__restrict__ sizes, const uint32_t *__restrict__ order, uint32_t n,
    const DevTables *__restrict__ tabs, const uint64_t *__restrict__ big_min_p,
    uint32_t *__restrict__ crc_out)
{
    __shared__ uint32_t sD[16 * 256];
    __shared__ uint32_t sT[256];
    constexpr int SV = 8;
    constexpr int NSETS = 2;
    constexpr uint32_t SB = 16 * SV;
    lds_fill(sD, &tabs->t.D[0][0], 16 * 256);
    lds_fill(sT, tabs->t.T, 256);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t wave0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
    if (wave0 >= n)
        return;
    const uint32_t i = wave0 + lane;
    bool valid = i < n;
    const uint32_t K16 = tabs->t.K16;
    const uint8_t *safe = reinterpret_cast<const uint8_t *>(tabs);  // >= 128 readable bytes
    uint32_t f = valid ? order[i] : 0;
    if (f >= n) {  // a stale order entry (the binning flagged it): no file
        valid = false;
        f = 0;
    }
    const uint64_t big_min = big_min_p ? *big_min_p : ~0ull;
    const uint64_t L0 = valid ? sizes[f] : 0;
    const bool mine = valid && L0 < big_min;  // else crc_seg_kernel's
    const uint64_t L = mine ? L0 : 0;
    const uint8_t *p = mine ? base + offs[f] : safe;
    uint32_t c = 0xFFFFFFFFu;  // CRC32_XINIT (storage/storage_service.c:7149)
    // the lane's geometry: bytes to 16-byte alignment, vectors to the line,
    // whole lines; recomputed after the steps (fewer registers live in them)
    struct Geo {
        uint64_t head, nvec, lead;
    };
    auto geo = [&]() {
        Geo g;
        g.head = (16u - ((uintptr_t)p & 15u)) & 15u;
        if (g.head > L)
            g.head = L;
        g.nvec = (L - g.head) >> 4;
        const uintptr_t va = (uintptr_t)(p + g.head);
        g.lead = ((SB - (va & (SB - 1))) & (SB - 1)) >> 4;
        if (g.lead > g.nvec)
            g.lead = g.nvec;
        return g;
    };
    uint32_t nsteps;
    {
        const Geo g = geo();
        for (uint64_t k = 0; k < g.head; k++)
            c = crc_byte<SAR>(sT, c, p[k]);
        const uint4 *v = reinterpret_cast<const uint4 *>(p + g.head);
        for (uint64_t j = 0; j < g.lead; j++)
            c = chain16<SAR>(sD, c, v[j], K16);
        nsteps = (uint32_t)((g.nvec - g.lead) / SV);
    }
    uint32_t nmax = nsteps;
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        const uint32_t y = __shfl_xor(nmax, o);
        nmax = y > nmax ? y : nmax;
    }
    if (nmax) {
        const uint4 *w = reinterpret_cast<const uint4 *>(p + geo().head) + geo().lead;
        uint32_t ring[32];
#pragma unroll
        for (int k = 0; k < 32; k++)
            ring[k] = 0;
        uint32_t zin = c ^ ((SAR && (int32_t)c < 0) ? tabs->t.Y4 : 0u);
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        auto ptr = [](u32x4 (&a)[SV], int q2) {
            uint32_t r0[4], r1[4], t[4];
#pragma unroll
            for (int d = 0; d < 4; d++) {
                r0[d] = a[2 * q2][d];
                r1[d] = a[2 * q2 + 1][d];
            }
            pair_transpose(r0, r1, t);
#pragma unroll
            for (int d = 0; d < 4; d++) {
                a[2 * q2][d] = r0[d];
                a[2 * q2 + 1][d] = t[d];
            }
        };
        auto step = [&](u32x4 (&a)[SV], bool ok) {
#pragma unroll
            for (int q = 0; q < SV; q++) {
                if ((q & 1) == 0) {
                    __builtin_amdgcn_sched_barrier(0);
                    ptr(a, q >> 1);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (ok) {
                    ring[4 * q + 0] = lane_fold_dw<SAR>(ring, 4 * q + 0, q == 0 ? a[q][0] ^ zin : a[q][0]);
                    ring[4 * q + 1] = lane_fold_dw<SAR>(ring, 4 * q + 1, a[q][1]);
                    ring[4 * q + 2] = lane_fold_dw<SAR>(ring, 4 * q + 2, a[q][2]);
                    ring[4 * q + 3] = lane_fold_dw<SAR>(ring, 4 * q + 3, a[q][3]);
                }
            }
            zin = 0;
        };
        u32x4 RS[NSETS][SV];
        // sig_hash_kernel's pair-cooperative loads (past-the-end steps read `safe`)
        auto issue_p = [&](u32x4 (&R)[SV], uint32_t stp) {
            const uint8_t *ln = stp < nsteps ? reinterpret_cast<const uint8_t *>(w + SV * (uint64_t)stp) : safe;
            const uint64_t a = reinterpret_cast<uint64_t>(ln);
            const uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
            auto ld = [&](int k, uint32_t lk, uint32_t hk) {
                const uint8_t *pk = reinterpret_cast<const uint8_t *>(((uint64_t)hk << 32 | lk) + 16u * (lane & 1));
                asm volatile("global_load_dwordx4 %0, %1, off offset:0" : "=v"(R[k]) : "v"(pk) : "memory");
                asm volatile("global_load_dwordx4 %0, %1, off offset:32" : "=v"(R[2 + k]) : "v"(pk) : "memory");
                asm volatile("global_load_dwordx4 %0, %1, off offset:64" : "=v"(R[4 + k]) : "v"(pk) : "memory");
                asm volatile("global_load_dwordx4 %0, %1, off offset:96" : "=v"(R[6 + k]) : "v"(pk) : "memory");
            };
#define PBC(S) (uint32_t) __builtin_amdgcn_mov_dpp((int)lo, S, 0xF, 0xF, false), \
               (uint32_t) __builtin_amdgcn_mov_dpp((int)hi, S, 0xF, 0xF, false)
            ld(0, PBC(0xA0));
            ld(1, PBC(0xF5));
#undef PBC
        };
        auto wait_older = [&](u32x4 (&R)[SV]) {
            asm volatile("s_waitcnt vmcnt(8)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]) :: "memory");
            asm volatile("" : "+v"(R[4]), "+v"(R[5]), "+v"(R[6]), "+v"(R[7]));
        };
        issue_p(RS[0], 0);
        for (uint32_t st = 0; st < nmax; st += NSETS) {
#pragma unroll
            for (int k = 0; k < NSETS; k++) {
                issue_p(RS[(k + 1) % NSETS], st + k + 1);
                wait_older(RS[k]);
                if (k == 0 || st + k < nmax)
                    step(RS[k], st + k < nsteps);
            }
        }
#pragma unroll
        for (int k = 0; k < NSETS; k++)
            asm volatile("s_waitcnt vmcnt(0)"
                         : "+v"(RS[k][0]), "+v"(RS[k][1]), "+v"(RS[k][2]), "+v"(RS[k][3]), "+v"(RS[k][4]),
                           "+v"(RS[k][5]), "+v"(RS[k][6]), "+v"(RS[k][7]) :: "memory");
        if (nsteps > 0)
            c = lane_fold_finish<SAR>(sD, K16, ring);
    }
    {
        const Geo g = geo();
        const uint4 *v = reinterpret_cast<const uint4 *>(p + g.head);
        for (uint64_t jv = g.lead + SV * (uint64_t)nsteps; jv < g.nvec; jv++)
            c = chain16<SAR>(sD, c, v[jv], K16);
        for (uint64_t k = g.head + (g.nvec << 4); k < L; k++)
            c = crc_byte<SAR>(sT, c, p[k]);
    }
    if (mine)
        crc_out[f] = c ^ 0xFFFFFFFFu;  // CRC32_FINAL (storage/storage_dio.c:500)
}

hipError_t launch_crc_lane(bool sar, const uint8_t *base, const uint64_t *offs, const uint64_t *sizes, uint32_t n,
                           const uint32_t *order, const DevTables *tabs, const uint64_t *big_min, uint32_t *crc_out,
                           hipStream_t st)
{
    const unsigned grid = (n + kHashBlock - 1) / kHashBlock;
    if (sar)
        crc_lane_kernel<true><<<grid, kHashBlock, 0, st>>>(base, offs, sizes, order, n, tabs, big_min, crc_out);
    else
        crc_lane_kernel<false><<<grid, kHashBlock, 0, st>>>(base, offs, sizes, order, n, tabs, big_min, crc_out);
    return hipGetLastError();
}

// simple_hash_ex / Time33Hash_ex of the big files (>= T), segment-parallel
// (INIT_HASH_CODES4 starts both at 0, so a file's hash is the polynomial
// sum_pos b_pos M^(L-1-pos) mod 2^32 and splits over any cut).  One wave per
// kSegBytes segment of the big-file list big_plan_kernel made; lane l hashes
// the segment's l-th 1/64 (Horner, 16-byte loads when the file is aligned),
// scales it by M^(bytes after it in the file) and the wave's sum is added
// into the file's slot (mod 2^32 addition commutes).  Multiplicative orders
// of 31 and 33 mod 2^32 divide 2^30, so exponents are reduced mod 2^30.
constexpr int kPolyBlock = 256;

__global__ __launch_bounds__(kPolyBlock) void poly_seg_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ boffs,
    const uint64_t *__restrict__ bsizes, const uint64_t *__restrict__ seg_first,
    const uint32_t *__restrict__ nbig, uint32_t *__restrict__ bpoly)
{
    const uint32_t nb = *nbig;
    const uint64_t total = seg_first[nb];
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * (kPolyBlock / 64);
    for (uint64_t sg = (uint64_t)blockIdx.x * (kPolyBlock / 64) + (threadIdx.x >> 6); sg < total; sg += nw) {
        uint32_t lo = 0, hi = nb;  // last file with seg_first <= sg
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (seg_first[mid] <= sg)
                lo = mid;
            else
                hi = mid;
        }
        const uint32_t f = lo;
        const uint64_t L = bsizes[f];
        const uint8_t *fp = base + boffs[f];
        constexpr uint64_t span = kSegBytes / 64;  // bytes per lane
        const uint64_t s0 = (sg - seg_first[f]) * kSegBytes + (uint64_t)lane * span;
        const uint64_t s1 = s0 + span < L ? s0 + span : L;
        uint32_t h31 = 0, h33 = 0;
        if (s0 < s1) {
            const uint8_t *q = fp + s0;
            uint64_t k = 0;
            const uint64_t len = s1 - s0;
            if ((((uintptr_t)q) & 15u) == 0) {
                for (; k + 16 <= len; k += 16) {
                    const uint4 v = *reinterpret_cast<const uint4 *>(q + k);
                    h31 = poly_word<31>(h31, v.x);
                    h33 = poly_word<33>(h33, v.x);
                    h31 = poly_word<31>(h31, v.y);
                    h33 = poly_word<33>(h33, v.y);
                    h31 = poly_word<31>(h31, v.z);
                    h33 = poly_word<33>(h33, v.z);
                    h31 = poly_word<31>(h31, v.w);
                    h33 = poly_word<33>(h33, v.w);
                }
            }
            for (; k < len; k++) {
                const uint32_t b = q[k];
                h31 = h31 * 31u + b;
                h33 = h33 * 33u + b;
            }
            const uint32_t e = (uint32_t)((L - s1) & 0x3FFFFFFFull);
            h31 *= pow_dev(31u, e);
            h33 *= pow_dev(33u, e);
        }
#pragma unroll
        for (int o = 32; o; o >>= 1) {
            h31 += __shfl_xor(h31, o);
            h33 += __shfl_xor(h33, o);
        }
        if (lane == 0) {
            atomicAdd(&bpoly[2ull * f], h31);
            atomicAdd(&bpoly[2ull * f + 1], h33);
        }
    }
}

hipError_t launch_poly_seg(const uint8_t *base, const uint64_t *boffs, const uint64_t *bsizes,
                           const uint64_t *seg_first, const uint32_t *nbig, uint32_t *bpoly,
                           unsigned grid, hipStream_t st)
{
    poly_seg_kernel<<<grid, kPolyBlock, 0, st>>>(base, boffs, bsizes, seg_first, nbig, bpoly);
    return hipGetLastError();
}

hipError_t launch_sig_hash(bool sar, const uint8_t *base, const uint64_t *offs,
                           const uint64_t *sizes, uint32_t n, const uint32_t *order,
                           const DevTables *tabs, const uint64_t *big_min, uint32_t *crc_out, uint8_t *sig_out,
                           int32_t *codes_out, fdfs_gpu_file_state *states, const uint32_t *sidx,
                           hipStream_t st, const uint32_t *nbig, uint32_t chain_cap)
{
    // the chain workgroups first: as many as there can be big files
    const uint32_t slots = (!nbig || !big_min) ? 0u : (n < chain_cap ? n : chain_cap);
    const unsigned grid = slots + (n + kHashBlock - 1) / kHashBlock;
#define HASH_LAUNCH(S, T)                                                                                \
    sig_hash_kernel<S, T><<<grid, kHashBlock, 0, st>>>(base, offs, sizes, order, n, tabs, big_min, crc_out, \
                                                       sig_out, codes_out, states, sidx, nbig, slots)
    if (states)
        sar ? HASH_LAUNCH(true, true) : HASH_LAUNCH(false, true);
    else
        sar ? HASH_LAUNCH(true, false) : HASH_LAUNCH(false, false);
#undef HASH_LAUNCH
    return hipGetLastError();
}

}  // namespace fdfs
