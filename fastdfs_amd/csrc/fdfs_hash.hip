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
//  * CRC32_ex: slice-by-16 byte tables in LDS (1 lookup per byte).
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

#include <cstdlib>

namespace fdfs {

// 256 threads: four workgroups (18 KB of tables each) per CU at 4 waves per
// SIMD; 512-thread workgroups ran 4 % slower (profiles/r01/hash_block_ab.txt).
constexpr int kHashBlock = 256;

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// All four CALC_HASH_CODES4 hashes of one 16-byte vector on the lane.
template <bool SAR, int TM>
__device__ __forceinline__ uint32_t crc16(const uint32_t *sD, const Rep8Lane &R8, uint32_t K,
                                          uint32_t c, uint4 q)
{
    if constexpr (TM == 2)
        return chain16r<SAR>(sD, R8, c, q, K);
    else
        return chain16<SAR>(sD, c, q, K);
}

template <bool SAR, int TM>
__device__ __forceinline__ void h4_lane(const uint32_t *sD, const Rep8Lane &R8, uint32_t K16,
                                        uint4 q, bool small, uint32_t &c, uint32_t &e, uint32_t &s,
                                        uint32_t &t)
{
    if (small)
        c = crc16<SAR, TM>(sD, R8, K16, c, q);
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

// ST (fdfs_gpu_update_batch): the lane continues the chunk's
// StorageFileContext-shaped state (crc32, file_hash_codes) instead of
// INIT_HASH_CODES4 and writes it back unfinalised; every step above is a
// recurrence from whatever state it starts in (the polynomial planes start
// from the lane's running value), so nothing else changes.
// Occupancy: the production instantiations fit four waves per SIMD (128
// registers) with AGPR accumulators as compiled.  Asking for four waves
// explicitly made hipcc move the ST form's accumulators to VGPRs (caught by
// tests/test_isa.py), so only the probe variant MODE 4 asks for it.
template <bool SAR, int TM, int MODE, bool ST, bool QL>
__global__ __launch_bounds__(TM == 2 || MODE == 5 ? 1024 : kHashBlock) __attribute__((amdgpu_waves_per_eu(MODE == 4 ? 4 : 1))) void sig_hash_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint64_t *__restrict__ sizes, const uint32_t *__restrict__ order, uint32_t n,
    const DevTables *__restrict__ tabs, const uint64_t *__restrict__ big_min_p,
    uint32_t *__restrict__ crc_out, uint8_t *__restrict__ sig_out, int32_t *__restrict__ codes_out,
    fdfs_gpu_file_state *__restrict__ states, const uint32_t *__restrict__ sidx)
{
    __shared__ uint32_t sD[TM == 2 ? kRep8Dwords : 16 * 256];
    __shared__ uint32_t sT[256];
    // SV vectors per step: 8 (one 128-byte line) or, probe MODE 6, 4 (half
    // a line: two 16-VGPR load sets instead of two of 32, and only B's last
    // four vectors in LDS)
    constexpr int SV = (MODE == 6 || MODE == 7) ? 4 : 8;
    // register sets of loads in flight: MODE 7 (probe) = four 64-byte sets,
    // the same 64 VGPRs as two 128-byte sets but 192 bytes of lookahead
    constexpr int NSETS = MODE == 7 ? 4 : 2;
    constexpr uint32_t SB = 16 * SV;  // bytes per step
    // 128-byte steps per Horner multiply of the accumulators (the B operands
    // then carry the coefficients of the whole group: fdfs_tables.hpp BG)
    constexpr int HG = SV == 8 ? kHornerGroup : 1;
    // The MFMA B operands, compacted: lane l's 16 bytes for (hash h, vector
    // q) are digit plane l & 3 of that vector's coefficients when l lies on
    // the block diagonal ((l >> 4) == ((l & 15) >> 2), fdfs_tables.cpp) and
    // zero otherwise -- five distinct 16-byte rows per (h, q): 1.25 KB of
    // LDS per step instead of 16 KB (rows 0-3 = lanes 0-3's B, row 4 = zero),
    // for the HG steps of a Horner group.
    __shared__ uint4 sB[2 * SV * HG * 5];
    if constexpr (TM == 2)
        lds_fill_rep8(sD, &tabs->t.D[0][0]);
    else
        lds_fill(sD, &tabs->t.D[0][0], 16 * 256);
    lds_fill(sT, tabs->t.T, 256);
    for (int i = threadIdx.x; i < 2 * SV * HG * 5; i += blockDim.x) {
        const int h = i / (SV * HG * 5), q = (i / 5) % (SV * HG), r = i % 5;
        const int8_t *row = HG > 1 ? &tabs->pm.BG[h][q][r & 3][0] : &tabs->pm.B[h][8 - SV + q][r & 3][0];
        sB[i] = r < 4 ? *reinterpret_cast<const uint4 *>(row) : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    const int brow = ((threadIdx.x & 63) >> 4) == ((threadIdx.x & 15) >> 2) ? (threadIdx.x & 3) : 4;

    const int lane = threadIdx.x & 63;
    const uint32_t wave0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
    if (wave0 >= n)  // whole wave past the batch (wave-uniform: MFMAs below need every lane)
        return;
    const uint32_t i = wave0 + lane;
    bool valid = i < n;
    const uint32_t K16 = TM == 2 ? tabs->t.K8 : tabs->t.K16;
    const Rep8Lane R8 = rep8_lane(lane);
    const uint8_t *safe = reinterpret_cast<const uint8_t *>(tabs);  // >= 128 readable bytes
    uint32_t f = valid ? order[i] : 0;
    if (f >= n) {  // a stale order entry (the binning flagged it): no file
        valid = false;
        f = 0;
    }
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
        h4_lane<SAR, TM>(sD, R8, K16, v[j], small, c, e, s, t);

    // whole steps: the wave steps in lockstep to its longest file
    const uint32_t nsteps = (uint32_t)((nvec - lead) / SV);
    uint32_t nmax = nsteps;
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        const uint32_t y = __shfl_xor(nmax, o);
        nmax = y > nmax ? y : nmax;
    }
    if (nmax) {
        const uint32_t m31 = SV == 8 ? tabs->pm.m1024[0] : tabs->pm.m64[0];
        const uint32_t m33 = SV == 8 ? tabs->pm.m1024[1] : tabs->pm.m64[1];
        const int col = lane & 15, j = col & 3, g = col >> 2;
        const int32_t kk31 = SV == 8 ? tabs->pm.KG[0][j] : tabs->pm.K64[0][j];
        const int32_t kk33 = SV == 8 ? tabs->pm.KG[1][j] : tabs->pm.K64[1][j];
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
        // QL: the step's pieces arrive interleaved over lane pairs (issue_p
        // below; probe MODE 15: over lane quads, issue_q) and are transposed
        // back to their files' lanes.
        auto qtr = [](u32x4 (&a)[SV], int h) {
#pragma unroll
            for (int d = 0; d < 4; d++) {
                uint32_t r0 = a[4 * h + 0][d], r1 = a[4 * h + 1][d], r2 = a[4 * h + 2][d], r3 = a[4 * h + 3][d];
                quad_transpose(r0, r1, r2, r3);
                a[4 * h + 0][d] = r0;
                a[4 * h + 1][d] = r1;
                a[4 * h + 2][d] = r2;
                a[4 * h + 3][d] = r3;
            }
        };
        // Pair-cooperative loads (issue_p; probe MODE 15: the round-2 quad
        // form, issue_q + qtr): one transpose stage per quarter line, just
        // before its two vectors are hashed.
        constexpr bool PAIR = MODE != 15;
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
                if (!mon || sg != 0 || MODE == 13)  // PROBE MODE 13: no Horner step (wrong results)
                    break;
                C31[r] = (int)((uint32_t)C31[r] * m31) + k31[r];
                C33[r] = (int)((uint32_t)C33[r] * m33) + k33[r];
            }
#pragma unroll
            for (int q = 0; q < SV; q++) {
                if constexpr (QL && PAIR && MODE != 1) {
                    if ((q & 1) == 0) {
                        __builtin_amdgcn_sched_barrier(0);
                        ptr(a, q >> 1);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                } else if constexpr (QL && MODE != 1) {
                    if ((q & 3) == 0) {
                        __builtin_amdgcn_sched_barrier(0);
                        qtr(a, q >> 2);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
                const uint4 aq = make_uint4(a[q][0], a[q][1], a[q][2], a[q][3]);
                if constexpr (MODE == 1) {  // PROBE: loads only
                    if (ok)
                        c ^= aq.x ^ aq.y ^ aq.z ^ aq.w;
                    continue;
                }
                if constexpr (MODE == 3 && TM == 0) {  // PROBE: CRC lookups, ELF, then the CRC XOR tree
                    if (ok) {
                        uint32_t v[16];
                        if (small)
                            chain16_issue(sD, c, aq, v);
                        __builtin_amdgcn_sched_barrier(0);
                        elf_word4<SAR, false>(aq.x, e);
                        elf_word4<SAR, false>(aq.y, e);
                        elf_word4<SAR, false>(aq.z, e);
                        elf_word4<SAR, true>(aq.w, e);
                        __builtin_amdgcn_sched_barrier(0);
                        if (small)
                            c = chain16_finish<SAR>(v, c, K16);
                    }
                } else if constexpr (MODE == 4) {  // PROBE: ELF in the 3-op chain form
                    if (ok) {
                        if (small)
                            c = crc16<SAR, TM>(sD, R8, K16, c, aq);
                        elf_word4_chain<SAR, false>(aq.x, e);
                        elf_word4_chain<SAR, false>(aq.y, e);
                        elf_word4_chain<SAR, false>(aq.z, e);
                        elf_word4_chain<SAR, true>(aq.w, e);
                    }
                } else if (ok) {
                    // PROBE ablations (wrong results): MODE 10 no ELF, MODE 11 no CRC
                    if (small && MODE != 11)
                        c = crc16<SAR, TM>(sD, R8, K16, c, aq);
                    if constexpr (MODE != 10) {
                        // the top nibble stays dirty across vectors (each
                        // step shifts it out); made exact once after the
                        // steps from the last t's sign (elf_exact_after)
                        elf_vec16y<SAR>(aq, e, ylast);
                    } else {
                        e += aq.x ^ aq.y ^ aq.z ^ aq.w;
                    }
                }
                if (!mon || MODE == 9)  // PROBE MODE 9: no MFMA planes (wrong results)
                    continue;
                // b - 128 as int8 (b ^ 0x80); a padded step is all-zero data
                const uint32_t msk = ok ? 0xFFFFFFFFu : 0u;
                const i32x4 A = {(int)and_xor80(aq.x, msk), (int)and_xor80(aq.y, msk),
                                 (int)and_xor80(aq.z, msk), (int)and_xor80(aq.w, msk)};
                // the step's vector q carries coefficients M^(SB-1-pos): B's vectors 8 - SV + q
                const uint4 b31 = sB[(0 * SV * HG + sg * SV + q) * 5 + brow];
                const uint4 b33 = sB[(1 * SV * HG + sg * SV + q) * 5 + brow];
                const i32x4 B31 = {(int)b31.x, (int)b31.y, (int)b31.z, (int)b31.w};
                const i32x4 B33 = {(int)b33.x, (int)b33.y, (int)b33.z, (int)b33.w};
                C31 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B31, C31, 0, 0, 0);
                C33 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B33, C33, 0, 0, 0);
            }
        };
        // The next step's line is loaded while this one is hashed: two
        // register sets, asm loads (hipcc would sink plain loads to their
        // use), issued unconditionally (past-the-end steps read `safe`) so no
        // register an asm load is still writing is ever copied.
        u32x4 RS[NSETS][SV];
        auto issue = [&](u32x4 (&R)[SV], uint32_t stp) {
            const uint8_t *ln = (MODE != 2 && stp < nsteps) ? reinterpret_cast<const uint8_t *>(w + SV * (uint64_t)stp) : safe;
#pragma unroll
            for (int q = 0; q < SV; q++)
                asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(R[q]) : "v"(ln), "i"(16 * q) : "memory");
        };
        // Quad-cooperative form (probe MODE 15, production in rounds 2-4):
        // lane j of quad Q loads 16-byte piece 4h + j of quad-file k's line
        // into R[4h + k], so each instruction reads 16 half lines of 64
        // contiguous bytes instead of 64 scattered 16-byte pieces (loads alone
        // 6.8 -> 6.0 ms on config 2, profiles/r02/hash_quad_ab.md), at 8 VALU
        // of transposes per vector.  MODE 12 (non-temporal) was measured on
        // this form.  The quad's line addresses are broadcast by DPP quad_perm.
        auto issue_q = [&](u32x4 (&R)[SV], uint32_t stp) {
            const uint8_t *ln = (MODE != 2 && stp < nsteps) ? reinterpret_cast<const uint8_t *>(w + SV * (uint64_t)stp) : safe;
            const uint64_t a = reinterpret_cast<uint64_t>(ln);
            const uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
            auto ld = [&](int k, uint32_t lk, uint32_t hk) {
                const uint8_t *pk = reinterpret_cast<const uint8_t *>(((uint64_t)hk << 32 | lk) + 16u * (lane & 3));
                if constexpr (MODE == 12) {  // PROBE: non-temporal loads
                    asm volatile("global_load_dwordx4 %0, %1, off offset:0 nt" : "=v"(R[k]) : "v"(pk) : "memory");
                    asm volatile("global_load_dwordx4 %0, %1, off offset:64 nt" : "=v"(R[k + 4]) : "v"(pk) : "memory");
                } else {
                    asm volatile("global_load_dwordx4 %0, %1, off offset:0" : "=v"(R[k]) : "v"(pk) : "memory");
                    if constexpr (SV == 8)
                        asm volatile("global_load_dwordx4 %0, %1, off offset:64" : "=v"(R[k + 4]) : "v"(pk) : "memory");
                }
            };
#define QBC(K) (uint32_t) __builtin_amdgcn_mov_dpp((int)lo, 0x55 * K, 0xF, 0xF, false), \
               (uint32_t) __builtin_amdgcn_mov_dpp((int)hi, 0x55 * K, 0xF, 0xF, false)
            ld(0, QBC(0));
            ld(1, QBC(1));
            ld(2, QBC(2));
            ld(3, QBC(3));
#undef QBC
        };
        // Pair-cooperative form (production since round 4): lane j of pair P
        // loads piece 2p + j of pair-file k's line into R[2p + k]: 32
        // contiguous bytes per lane pair per instruction, one transpose stage
        // (4 VALU per vector instead of the quad form's 8): 8.41 against
        // 8.58-8.60 ms (profiles/r04/pair_loads_ab.txt).  The pair's line
        // addresses are broadcast by DPP quad_perm [k,k,2+k,2+k].
        auto issue_p = [&](u32x4 (&R)[SV], uint32_t stp) {
            const uint8_t *ln = (MODE != 2 && stp < nsteps) ? reinterpret_cast<const uint8_t *>(w + SV * (uint64_t)stp) : safe;
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
            if constexpr (SV == 8) {
                static_assert(NSETS == 2, "128-byte steps: two sets");
                asm volatile("s_waitcnt vmcnt(8)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]) :: "memory");
                asm volatile("" : "+v"(R[4]), "+v"(R[5]), "+v"(R[6]), "+v"(R[7]));
            } else if constexpr (NSETS == 4) {
                asm volatile("s_waitcnt vmcnt(12)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]) :: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(4)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]) :: "memory");
            }
        };
        auto drain = [&]() {
#pragma unroll
            for (int k = 0; k < NSETS; k++) {
                if constexpr (SV == 8) {
                    asm volatile("s_waitcnt vmcnt(0)"
                                 : "+v"(RS[k][0]), "+v"(RS[k][1]), "+v"(RS[k][2]), "+v"(RS[k][3]), "+v"(RS[k][4]),
                                   "+v"(RS[k][5]), "+v"(RS[k][6]), "+v"(RS[k][7]) :: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" : "+v"(RS[k][0]), "+v"(RS[k][1]), "+v"(RS[k][2]), "+v"(RS[k][3]) :: "memory");
                }
            }
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
        if (nfull) {
            auto iss = [&](u32x4 (&R)[SV], uint32_t stp) {
                // probe MODE 8: the step's loads issued at raised wave
                // priority, so they leave ahead of the other waves' VALU
                if constexpr (MODE == 8)
                    __builtin_amdgcn_s_setprio(2);
                if constexpr (QL && PAIR)
                    issue_p(R, stp);
                else if constexpr (QL)
                    issue_q(R, stp);
                else
                    issue(R, stp);
                if constexpr (MODE == 8)
                    __builtin_amdgcn_s_setprio(0);
            };
            pipeline(iss, step, 0u, nfull);
        }
        // The rest of the steps (waves of big files: ELF alone, its
        // dependent chain the bound).  Four 64-byte load sets here (192 B of
        // lookahead in the same registers) measured 906-962 against 826-940
        // ms on config 1, within that config's run-to-run spread
        // (profiles/r03/hash_pipeline_ab.txt): not kept.
        auto step_chain = [&](u32x4 (&a)[SV], bool ok, uint32_t) {
            if (MODE == 1 || !ok)
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
        s = s31 * pow_dev(SV == 8 ? tabs->pm.inv128[0] : tabs->pm.inv64[0], pad);
        t = s33 * pow_dev(SV == 8 ? tabs->pm.inv128[1] : tabs->pm.inv64[1], pad);
    }

    for (uint64_t jv = lead + SV * (uint64_t)nsteps; jv < nvec; jv++)
        h4_lane<SAR, TM>(sD, R8, K16, v[jv], small, c, e, s, t);
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

#ifdef FDFS_PROBES  // measured, not kept: the probe build only
// ---------------------------------------------------------------------------
// sig_split_kernel: the role-split form of sig_hash_kernel (VERDICT r03 item
// 2).  A 1024-thread workgroup per CU: waves 0-3 are loaders (one per SIMD:
// a workgroup's waves are dealt to the SIMDs cyclically), waves 4-15 hash
// 12 x 64 files of the size-sorted order.  Every 128-byte step ("round") of
// the 768 files: each loader has its three hash waves' lines in registers
// (24 x 16 B per lane, cooperative: 8 lanes read one file's whole line, one
// load instruction reads the lines of 8 files), writes them to one LDS row
// per file (144-byte stride: ds_write_b128 and ds_read_b128 conflict-free),
// and issues the next round's loads; the hash waves read their rows and run
// CRC (slice-by-16), ELF and the MFMA polynomial planes exactly as
// sig_hash_kernel's step does -- but never wait on HBM, carry no load
// registers and no quad transposes.  Two barriers per round (rows full, rows
// read), lgkmcnt only, so the loaders' next loads stay in flight across them;
// the 768 files of a workgroup are consecutive in the size order (near-equal
// sizes), so the lockstep costs little.  Bound (profiles/r04/probes_r04b.txt):
// the compute-only hash kernel at three waves per SIMD without transposes
// takes 6.22 ms on config 2, the loads alone ~6.1 ms, sig_hash_kernel 8.8 ms.
// The head (to 16-byte alignment), lead (to 128-byte alignment) and tail
// bytes are lane-serial from global memory, as in sig_hash_kernel, so the
// loaders' lines are whole aligned 128-byte lines.
// chain16 with the XORs as __builtin_amdgcn_bitop3_b32 instead of the xor3
// asm statement: the split kernel's hash loop holds no inline asm at all, so
// hipcc sees every instruction between its MFMAs and pads every hazard itself
// (its accumulators are VGPRs: a 1024-thread workgroup leaves 128 registers
// per wave, and hipcc then picks the VGPR form of the MFMAs).
template <bool SAR>
__device__ __forceinline__ uint32_t chain16_b(const uint32_t *__restrict__ D, uint32_t c, uint4 w, uint32_t K16)
{
    auto x3 = [](uint32_t a, uint32_t b, uint32_t d) { return __builtin_amdgcn_bitop3_b32(a, b, d, 0x96); };
    const uint32_t x = c ^ w.x;
    uint32_t r0 = x3(D[0 * 256 + (x & 0xFFu)], D[1 * 256 + ((x >> 8) & 0xFFu)], D[2 * 256 + ((x >> 16) & 0xFFu)]);
    uint32_t r1 = x3(D[3 * 256 + (x >> 24)], D[4 * 256 + (w.y & 0xFFu)], D[5 * 256 + ((w.y >> 8) & 0xFFu)]);
    uint32_t r2 = x3(D[6 * 256 + ((w.y >> 16) & 0xFFu)], D[7 * 256 + (w.y >> 24)], D[8 * 256 + (w.z & 0xFFu)]);
    uint32_t r3 = x3(D[9 * 256 + ((w.z >> 8) & 0xFFu)], D[10 * 256 + ((w.z >> 16) & 0xFFu)], D[11 * 256 + (w.z >> 24)]);
    r0 = x3(r0, D[12 * 256 + (w.w & 0xFFu)], D[13 * 256 + ((w.w >> 8) & 0xFFu)]);
    r1 = x3(r1, D[14 * 256 + ((w.w >> 16) & 0xFFu)], D[15 * 256 + (w.w >> 24)]);
    uint32_t r = x3(r0, r1, r2) ^ r3;
    if (SAR)
        r ^= (uint32_t)((int32_t)c >> 31) & K16;
    return r;
}

constexpr int kSplitHash = 12;                     // hash waves per workgroup
constexpr int kSplitLoad = 4;                      // loader waves
constexpr int kSplitThreads = 64 * (kSplitHash + kSplitLoad);
constexpr uint32_t kSplitFiles = 64 * kSplitHash;  // files per workgroup
constexpr int kSplitRow = 144;                     // LDS row stride (128 B + 16 pad)
static_assert(kSplitHash == 3 * kSplitLoad, "each loader serves three hash waves");

__device__ __forceinline__ void split_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <bool SAR>
__global__ __launch_bounds__(kSplitThreads) void sig_split_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint64_t *__restrict__ sizes, const uint32_t *__restrict__ order, uint32_t n,
    const DevTables *__restrict__ tabs, const uint64_t *__restrict__ big_min_p,
    uint32_t *__restrict__ crc_out, uint8_t *__restrict__ sig_out, int32_t *__restrict__ codes_out)
{
    constexpr int SV = 8;
    __shared__ uint32_t sD[16 * 256];
    __shared__ uint32_t sT[256];
    __shared__ uint4 sB[2 * SV * 64];
    __shared__ __attribute__((aligned(16))) uint8_t rows[kSplitHash][64 * kSplitRow];
    __shared__ ulonglong2 wins[kSplitFiles];  // per file: {first line, end of the last whole line}
    __shared__ uint32_t s_nround;
    lds_fill(sD, &tabs->t.D[0][0], 16 * 256);
    lds_fill(sT, tabs->t.T, 256);
#pragma unroll
    for (int h = 0; h < 2; h++)
        lds_fill(reinterpret_cast<uint32_t *>(sB + h * SV * 64),
                 reinterpret_cast<const uint32_t *>(&tabs->pm.B[h][0][0][0]), SV * 64 * 4);
    if (threadIdx.x == 0)
        s_nround = 0;
    __syncthreads();

    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint8_t *safe = reinterpret_cast<const uint8_t *>(tabs);  // >= 128 readable bytes
    const uint32_t f0 = blockIdx.x * kSplitFiles;

    if (wv < kSplitLoad) {  // ---------------------------------------- loader
        split_barrier();  // the hash waves' windows are in `wins`
        const uint32_t nround = s_nround;
        const int piece = lane & 7, fsub = lane >> 3;
        u32x4 R[3][8];
        auto issue = [&](uint32_t r) {
#pragma unroll
            for (int j = 0; j < 3; j++) {
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const ulonglong2 wd = wins[(wv + kSplitLoad * j) * 64 + 8 * k + fsub];
                    const uint64_t a = wd.x + 128ull * r;
                    const uint8_t *ln = (a < wd.y ? reinterpret_cast<const uint8_t *>(a) : safe) + 16 * piece;
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(R[j][k]) : "v"(ln) : "memory");
                }
            }
        };
        if (nround)
            issue(0);
        for (uint32_t r = 0; r < nround; r++) {
            asm volatile("s_waitcnt vmcnt(0)"
                         : "+v"(R[0][0]), "+v"(R[0][1]), "+v"(R[0][2]), "+v"(R[0][3]), "+v"(R[0][4]),
                           "+v"(R[0][5]), "+v"(R[0][6]), "+v"(R[0][7]), "+v"(R[1][0]), "+v"(R[1][1]),
                           "+v"(R[1][2]), "+v"(R[1][3]), "+v"(R[1][4]), "+v"(R[1][5]), "+v"(R[1][6]),
                           "+v"(R[1][7]), "+v"(R[2][0]), "+v"(R[2][1]), "+v"(R[2][2]), "+v"(R[2][3]),
                           "+v"(R[2][4]), "+v"(R[2][5]), "+v"(R[2][6]), "+v"(R[2][7])
                         :: "memory");
#pragma unroll
            for (int j = 0; j < 3; j++) {
                uint8_t *tile = rows[wv + kSplitLoad * j];
#pragma unroll
                for (int k = 0; k < 8; k++)
                    *reinterpret_cast<u32x4 *>(tile + (8 * k + fsub) * kSplitRow + 16 * piece) = R[j][k];
            }
            split_barrier();  // X: rows of round r full (and R free: lgkmcnt(0))
            if (r + 1 < nround)
                issue(r + 1);
            split_barrier();  // Y: the hash waves have read round r
        }
        return;
    }

    // ------------------------------------------------------------------ hash
    const int hw = wv - kSplitLoad;
    const uint32_t i = f0 + hw * 64 + lane;
    bool valid = i < n;
    const uint32_t K16 = tabs->t.K16;
    const Rep8Lane R8 = rep8_lane(lane);  // unused by the TM 0 tables
    uint32_t f = valid ? order[i] : 0;
    if (f >= n) {  // a stale order entry (the binning flagged it): no file
        valid = false;
        f = 0;
    }
    const uint64_t L = valid ? sizes[f] : 0;
    const uint8_t *p = valid ? base + offs[f] : safe;
    uint32_t c = 0xFFFFFFFFu;      // CRC32_XINIT (storage/storage_service.c:7149)
    uint32_t e = 0, s = 0, t = 0;  // INIT_HASH_CODES4 (storage/storage_service.c:7156)
    const uint64_t big_min = big_min_p ? *big_min_p : ~0ull;
    const bool small = L < big_min;
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
    uint64_t lead = ((128u - ((uintptr_t)v & 127u)) & 127u) >> 4;
    if (lead > nvec)
        lead = nvec;
    for (uint64_t j = 0; j < lead; j++)
        h4_lane<SAR, 0>(sD, R8, K16, v[j], small, c, e, s, t);
    const uint32_t nsteps = (uint32_t)((nvec - lead) / SV);
    {
        const uint64_t w0 = reinterpret_cast<uint64_t>(v + lead);
        wins[hw * 64 + lane] = make_ulonglong2(w0, w0 + 128ull * nsteps);
    }
    uint32_t nmax = nsteps, nfull = small ? nsteps : 0;
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        const uint32_t y = __shfl_xor(nmax, o), z = __shfl_xor(nfull, o);
        nmax = y > nmax ? y : nmax;
        nfull = z > nfull ? z : nfull;
    }
    if (lane == 0)
        atomicMax(&s_nround, nmax);
    split_barrier();
    const uint32_t nround = s_nround;

    const uint32_t m31 = tabs->pm.m128[0], m33 = tabs->pm.m128[1];
    const int col = lane & 15, jj = col & 3, g = col >> 2;
    const int32_t kk31 = tabs->pm.K[0][jj], kk33 = tabs->pm.K[1][jj];
    const i32x4 k31 = {kk31, kk31, kk31, kk31};
    const i32x4 k33 = {kk33, kk33, kk33, kk33};
    i32x4 C31 = {0, 0, 0, 0}, C33 = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int src = 16 * g + 4 * (lane >> 4) + r;
        const uint32_t s0 = __shfl(s, src), t0 = __shfl(t, src);
        C31[r] = jj == 0 ? (int)s0 : 0;
        C33[r] = jj == 0 ? (int)t0 : 0;
    }
    uint32_t nexec = 0;
    const uint8_t *mine = rows[hw] + lane * kSplitRow;
    for (uint32_t r = 0; r < nround; r++) {
        split_barrier();  // X: round r's rows are in LDS
        uint4 a[SV];
        if (r < nmax) {
#pragma unroll
            for (int q = 0; q < SV; q++)
                a[q] = *reinterpret_cast<const uint4 *>(mine + 16 * q);
        }
        split_barrier();  // Y: rows read (lgkmcnt(0)); the loaders may refill
        if (r >= nmax)
            continue;
        const bool ok = r < nsteps;
        if (r < nfull) {
            const bool mon = __any(ok && small);
            nexec += mon ? 1u : 0u;
            if (mon) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    C31[k] = (int)((uint32_t)C31[k] * m31) + k31[k];
                    C33[k] = (int)((uint32_t)C33[k] * m33) + k33[k];
                }
            }
#pragma unroll
            for (int q = 0; q < SV; q++) {
                const uint4 aq = a[q];
                if (ok) {  // no inline asm here (see chain16_b)
                    if (small)
                        c = chain16_b<SAR>(sD, c, aq, K16);
                    elf_word4_chain<SAR, false>(aq.x, e);
                    elf_word4_chain<SAR, false>(aq.y, e);
                    elf_word4_chain<SAR, false>(aq.z, e);
                    elf_word4_chain<SAR, true>(aq.w, e);
                }
                if (!mon)
                    continue;
                const uint32_t msk = ok ? 0xFFFFFFFFu : 0u;
                const i32x4 A = {(int)and_xor80(aq.x, msk), (int)and_xor80(aq.y, msk),
                                 (int)and_xor80(aq.z, msk), (int)and_xor80(aq.w, msk)};
                const uint4 b31 = sB[(0 * SV + q) * 64 + lane], b33 = sB[(1 * SV + q) * 64 + lane];
                const i32x4 B31 = {(int)b31.x, (int)b31.y, (int)b31.z, (int)b31.w};
                const i32x4 B33 = {(int)b33.x, (int)b33.y, (int)b33.z, (int)b33.w};
                C31 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B31, C31, 0, 0, 0);
                C33 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B33, C33, 0, 0, 0);
            }
        } else if (ok) {  // waves of big files past their small lanes: ELF alone
#pragma unroll
            for (int q = 0; q < SV; q++) {
                elf_word4_chain<SAR, false>(a[q].x, e);
                elf_word4_chain<SAR, false>(a[q].y, e);
                elf_word4_chain<SAR, false>(a[q].z, e);
                elf_word4_chain<SAR, true>(a[q].w, e);
            }
        }
    }
    if (nmax) {  // planes -> value, back to the file's lane, padded steps undone
        uint32_t s31 = 0, s33 = 0;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            uint32_t x = (uint32_t)C31[r] << (8 * jj), y = (uint32_t)C33[r] << (8 * jj);
            x += __shfl_xor(x, 1);
            y += __shfl_xor(y, 1);
            x += __shfl_xor(x, 2);
            y += __shfl_xor(y, 2);
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
        h4_lane<SAR, 0>(sD, R8, K16, v[jv], small, c, e, s, t);
    for (uint64_t k = head + (nvec << 4); k < L; k++) {  // the last (L - head) & 15 bytes
        const uint32_t b = p[k];
        if (small)
            c = crc_byte<SAR>(sT, c, b);
        h3_byte<SAR>(b, e, s, t);
    }
    if (!valid)
        return;
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
#endif

// simple_hash_ex / Time33Hash_ex of the big files (>= T), segment-parallel
// (INIT_HASH_CODES4 starts both at 0, so a file's hash is the polynomial
// sum_pos b_pos M^(L-1-pos) mod 2^32 and splits over any cut).  One wave per
// 64 KiB segment of the big-file list big_plan_kernel made; lane l hashes
// the segment's l-th KiB (Horner, 16-byte loads when the file is aligned),
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
        const uint64_t s0 = (sg - seg_first[f]) * kSegBytes + (uint64_t)lane * 1024;
        const uint64_t s1 = s0 + 1024 < L ? s0 + 1024 : L;
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
                           hipStream_t st)
{
#ifdef FDFS_PROBES
    // measurement build only (make probes): FDFS_GPU_HASH_MODE 1 = loads
    // only, 2 = compute only (wrong results), 3 = CRC lookups / ELF / CRC
    // XOR tree in that order, 4 = ELF in the 3-op chain form, 5 = production
    // code in 1024-thread workgroups, 6 = 64-byte steps, 7 = 64-byte steps
    // with four load sets in flight, 8 = loads issued at raised priority;
    // FDFS_GPU_HASH_TM CRC table form
    // 0 = slice-by-16 bytes, 2 = rotated rep8
    static int mode = -1;
    if (mode < 0) {
        const char *ev = getenv("FDFS_GPU_HASH_MODE");
        mode = ev ? atoi(ev) : 0;
    }
    static int tm = -1;
    if (tm < 0) {
        const char *ev = getenv("FDFS_GPU_HASH_TM");
        tm = ev ? atoi(ev) : 0;
    }
#else
    [[maybe_unused]] constexpr int tm = 0;
    [[maybe_unused]] constexpr int mode = 0;
#endif
#ifdef FDFS_PROBES
    static int ql = -1;  // FDFS_GPU_HASH_QUAD=0: round-2 lane-per-file loads
    if (ql < 0) {
        const char *ev = getenv("FDFS_GPU_HASH_QUAD");
        ql = ev ? atoi(ev) : 1;
    }
#else
    constexpr int ql = 1;
#endif
#ifdef FDFS_PROBES
    const unsigned blk0 = ((tm >= 2 || mode == 5) && !states) ? 1024 : kHashBlock;
    // FDFS_GPU_HASH_LDSPAD: dynamic LDS bytes per workgroup that the kernel
    // does not use, to cap its occupancy (waves per SIMD) for the role-split
    // bound of DESIGN 4.2
    static long shm = -1;
    if (shm < 0) {
        const char *ev = getenv("FDFS_GPU_HASH_LDSPAD");
        shm = ev ? atol(ev) : 0;
    }
    static int hb = -1;  // FDFS_GPU_HASH_BLOCK: workgroup size (the LDS now fits eight per CU)
    if (hb < 0) {
        const char *ev = getenv("FDFS_GPU_HASH_BLOCK");
        hb = ev ? atoi(ev) : 0;
    }
    const unsigned blk = hb == 128 || hb == 64 || (hb == 512 && !states) ? (unsigned)hb : blk0;
#else
    const unsigned blk = kHashBlock;
    constexpr unsigned shm = 0;
#endif
    const unsigned grid = (n + blk - 1) / blk;
#ifdef FDFS_PROBES
    static int split = -1;  // FDFS_GPU_HASH_SPLIT=1: the role-split kernel (one-shot batches)
    if (split < 0) {
        const char *ev = getenv("FDFS_GPU_HASH_SPLIT");
        split = ev ? atoi(ev) : 0;
    }
#endif
#ifdef FDFS_PROBES
    if (split && !states && mode == 0 && tm == 0) {
        const unsigned g2 = (n + kSplitFiles - 1) / kSplitFiles;
        if (sar)
            sig_split_kernel<true><<<g2, kSplitThreads, 0, st>>>(base, offs, sizes, order, n, tabs, big_min, crc_out,
                                                               sig_out, codes_out);
        else
            sig_split_kernel<false><<<g2, kSplitThreads, 0, st>>>(base, offs, sizes, order, n, tabs, big_min, crc_out,
                                                                sig_out, codes_out);
        return hipGetLastError();
    }
#endif
#ifdef FDFS_PROBES
#define HASH_LAUNCH_TM2(S, M)                                                                            \
    else if (tm == 2)                                                                                    \
        sig_hash_kernel<S, 2, M, false, false><<<grid, blk, (unsigned)shm, st>>>(base, offs, sizes, order, n, tabs, big_min, \
                                                                     crc_out, sig_out, codes_out, nullptr, nullptr); \
    else if (tm == 3)                                                                                    \
        sig_hash_kernel<S, 2, M, false, true><<<grid, blk, (unsigned)shm, st>>>(base, offs, sizes, order, n, tabs, big_min, \
                                                                    crc_out, sig_out, codes_out, nullptr, nullptr);
#else
// the rotated-table form (TM 2, VGPR accumulators) exists in the probe
// build only: the production library holds AGPR-accumulator kernels alone
// (tests/test_isa.py)
#define HASH_LAUNCH_TM2(S, M)
#endif
#define HASH_LAUNCH(S, M)                                                                                \
    do {                                                                                                 \
        if (states)                                                                                      \
            sig_hash_kernel<S, 0, M, true, true><<<grid, blk, (unsigned)shm, st>>>(base, offs, sizes, order, n, tabs, big_min, \
                                                                 crc_out, sig_out, codes_out, states, sidx); \
        HASH_LAUNCH_TM2(S, M)                                                                            \
        else if (ql)                                                                                     \
            sig_hash_kernel<S, 0, M, false, true><<<grid, blk, (unsigned)shm, st>>>(base, offs, sizes, order, n, tabs, big_min, \
                                                                  crc_out, sig_out, codes_out, nullptr, nullptr); \
        else                                                                                             \
            sig_hash_kernel<S, 0, M, false, false><<<grid, blk, (unsigned)shm, st>>>(base, offs, sizes, order, n, tabs, big_min, \
                                                                  crc_out, sig_out, codes_out, nullptr, nullptr); \
    } while (0)
#ifdef FDFS_PROBES
    if (mode == 1)
        HASH_LAUNCH(true, 1);
    else if (mode == 2)
        HASH_LAUNCH(true, 2);
    else if (mode == 3)
        HASH_LAUNCH(true, 3);
    else if (mode == 4)
        HASH_LAUNCH(true, 4);
    else if (mode == 5)  // production code in 1024-thread workgroups (the TM 2/3 block size)
        HASH_LAUNCH(true, 5);
    else if (mode == 6)  // 64-byte steps: two 16-VGPR load sets
        HASH_LAUNCH(true, 6);
    else if (mode == 7)  // 64-byte steps: four 16-VGPR load sets (192 bytes ahead)
        HASH_LAUNCH(true, 7);
    else if (mode == 8)  // the step's loads issued at s_setprio 2
        HASH_LAUNCH(true, 8);
    else if (((mode >= 9 && mode <= 13) || mode == 15) && !states && ql) {  // ablations: no MFMA / no ELF / no CRC / no Horner; nt loads; quad loads
        if (mode == 15 && !sar)
            sig_hash_kernel<false, 0, 15, false, true><<<grid, blk, (unsigned)shm, st>>>(
                base, offs, sizes, order, n, tabs, big_min, crc_out, sig_out, codes_out, nullptr, nullptr);
        else if (mode == 15)
            sig_hash_kernel<true, 0, 15, false, true><<<grid, blk, (unsigned)shm, st>>>(
                base, offs, sizes, order, n, tabs, big_min, crc_out, sig_out, codes_out, nullptr, nullptr);
        else if (mode == 13)
            sig_hash_kernel<true, 0, 13, false, true><<<grid, blk, (unsigned)shm, st>>>(
                base, offs, sizes, order, n, tabs, big_min, crc_out, sig_out, codes_out, nullptr, nullptr);
        else if (mode == 12 && !sar)
            sig_hash_kernel<false, 0, 12, false, true><<<grid, blk, (unsigned)shm, st>>>(
                base, offs, sizes, order, n, tabs, big_min, crc_out, sig_out, codes_out, nullptr, nullptr);
        else if (mode == 12)
            sig_hash_kernel<true, 0, 12, false, true><<<grid, blk, (unsigned)shm, st>>>(
                base, offs, sizes, order, n, tabs, big_min, crc_out, sig_out, codes_out, nullptr, nullptr);
        else if (mode == 9)
            sig_hash_kernel<true, 0, 9, false, true><<<grid, blk, (unsigned)shm, st>>>(
                base, offs, sizes, order, n, tabs, big_min, crc_out, sig_out, codes_out, nullptr, nullptr);
        else if (mode == 10)
            sig_hash_kernel<true, 0, 10, false, true><<<grid, blk, (unsigned)shm, st>>>(
                base, offs, sizes, order, n, tabs, big_min, crc_out, sig_out, codes_out, nullptr, nullptr);
        else
            sig_hash_kernel<true, 0, 11, false, true><<<grid, blk, (unsigned)shm, st>>>(
                base, offs, sizes, order, n, tabs, big_min, crc_out, sig_out, codes_out, nullptr, nullptr);
    } else
#endif
    if (sar)
        HASH_LAUNCH(true, 0);
    else
        HASH_LAUNCH(false, 0);
#undef HASH_LAUNCH
#undef HASH_LAUNCH_TM2
    return hipGetLastError();
}

}  // namespace fdfs
