// MD5 signature path (FDFS_SIG_MD5, file_signature_method=md5; config 3).
//
// Reference: my_md5_init / my_md5_update / my_md5_final (libfastcommon md5.c,
// RSA RFC 1321 code) driven by storage/storage_dio.c:480,512 and initialised
// at storage/storage_service.c:7160; the digest is the signature tail
// (storage/storage_service.c:106-120).
#include "fdfs_device.hpp"
#include "fdfs_kernels.hpp"
#include "fdfs_md5.hpp"
#include "fdfs_segcrc.hpp"

namespace fdfs {

__device__ __forceinline__ void store_sig(uint8_t *sig, uint64_t L, uint32_t w2, uint32_t w3,
                                          uint32_t w4, uint32_t w5)
{
    uint2 *sp = reinterpret_cast<uint2 *>(sig);
    sp[0] = make_uint2(bswap32((uint32_t)(L >> 32)), bswap32((uint32_t)L));
    sp[1] = make_uint2(w2, w3);
    sp[2] = make_uint2(w4, w5);
}

// Final block(s) of a file whose first nblk full 64-byte blocks are already
// folded into st: the L & 63 tail bytes at tp, 0x80, zero pad and the 64-bit
// bit length (RFC 1321 3.1-3.2; my_md5_final at storage/storage_dio.c:512).
__device__ __forceinline__ void md5_finish(uint32_t st[4], const uint8_t *tp, uint64_t L)
{
    const uint32_t r = (uint32_t)(L & 63u);
    uint32_t m[16];
#pragma unroll
    for (int wd = 0; wd < 16; wd++) {
        uint32_t word = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t k = 4 * wd + q;
            if (k < r)
                word |= (uint32_t)tp[k] << (8 * q);
        }
        m[wd] = word;
    }
    const uint64_t bits = L << 3;
    md5_pad_compress(st, m, r, (uint32_t)bits, (uint32_t)(bits >> 32));
}

// ------------------------------------------- MD5 path, one workgroup per file
//
// A batch's few big files (at most chain_cap of them: config 4's 1 GiB
// files) are each one serial chain, on one lane of one wave alone on its
// SIMD, and such a wave issues about one instruction per 4 cycles: every
// instruction it issues is time on the chain.  md5_compress spends five per
// step, one of them the a + m + K sum off the chain.  Here a helper wave makes
// those sums: its lane i computes K[i] + m[g(i)] of each block (g the RFC 1321
// message index of step i), a slot ahead of the MD5 wave (two slots of 32
// blocks in the tables' 16 KiB of LDS), which then runs four dependent
// instructions per step
// (md5_round_km) and reads each round's 16 sums one round ahead of its use.
// 16.8 against 21.2 cycles per byte on one wave (profiles/r06/
// chain_lds_ubench.json).  Every lane of the MD5 wave runs the same chain
// (the LDS reads broadcast); lane 0 stores.  The file's CRC comes from
// crc_seg_kernel (big_patch_kernel), as for any big file.
static __device__ const uint32_t kMd5Kc[64] = {
    0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u, 0xfd469501u,
    0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u, 0xa679438eu, 0x49b40821u,
    0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du, 0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u,
    0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu, 0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au,
    0xfffa3942u, 0x8771f681u, 0x6d9d6122u, 0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u,
    0x289b7ec6u, 0xeaa127fau, 0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u,
    0xf4292244u, 0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,
    0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu, 0xeb86d391u};

__device__ __forceinline__ int md5_msg_index(int i)  // g(i), RFC 1321 3.4
{
    return i < 16 ? i : i < 32 ? (5 * i + 1) & 15 : i < 48 ? (3 * i + 5) & 15 : (7 * i) & 15;
}

constexpr uint32_t kChainSlotBlocks = 32;  // blocks per LDS slot: 32 x 64 sums = 8 KiB

// ring: two slots, 16 KiB of the workgroup's LDS.  Every wave of the
// workgroup calls it: wave 0 runs the chain, wave 1 makes the sums, any
// others only keep the barrier count.  fs != nullptr: the state-carrying
// update (fdfs_gpu_update_batch): the chunk continues fs's MD5 -- the bytes
// my_md5_update left pending are completed first from the chunk's head, the
// chunk's last bytes become the new pending buffer, and the byte count
// advances (the CRC comes from big_patch_state_kernel).
__device__ __forceinline__ void md5_chain_wg(const uint8_t *p, uint64_t L, uint32_t f, int wv, uint4 *ring,
                                          uint8_t *sig_out, int32_t *codes_out, fdfs_gpu_file_state *fs)
{
    const int lane = threadIdx.x & 63;
    const uint32_t have = fs ? (fs->md5_count[0] >> 3) & 63u : 0u;  // bytes pending in fs's buffer
    const uint64_t pre = have ? (64 - have < L ? 64 - have : L) : 0;  // chunk bytes that complete them
    const uint8_t *s0 = p + pre;  // the stream of whole blocks
    const uint64_t nblk = (L - pre) >> 6;
    const uint64_t nslots = uniform64((nblk + kChainSlotBlocks - 1) / kChainSlotBlocks);
    if (wv == 1) {
        const uint32_t kk = kMd5Kc[lane];
        const uint8_t *src = s0 + 4 * md5_msg_index(lane);
        auto fill = [&](uint4 *slot, uint64_t s) {
            const uint64_t b0 = s * kChainSlotBlocks;
            const uint32_t nb = (uint32_t)uniform64(nblk - b0 < kChainSlotBlocks ? nblk - b0 : kChainSlotBlocks);
            uint32_t *w = reinterpret_cast<uint32_t *>(slot);
            for (uint32_t j0 = 0; j0 < nb; j0 += 16) {
                uint32_t v[16];
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const uint64_t blk = b0 + j0 + u < nblk ? b0 + j0 + u : b0;  // past the end: re-read block b0
                    __builtin_memcpy(&v[u], src + 64 * blk, 4);  // any alignment (unaligned memory mode)
                }
#pragma unroll
                for (int u = 0; u < 16; u++)
                    w[(j0 + u) * 64 + lane] = v[u] + kk;
            }
        };
        if (nslots)
            fill(ring, 0);
        __syncthreads();
        for (uint64_t s = 0; s < nslots; s++) {
            if (s + 1 < nslots)
                fill(ring + ((s + 1) & 1) * (kChainSlotBlocks * 16), s + 1);
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
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};  // my_md5_init
    if (fs) {
#pragma unroll
        for (int k = 0; k < 4; k++)
            st[k] = fs->md5_state[k];
        if (have && have + pre == 64) {  // my_md5_update's partial block: buffer || chunk head
            uint32_t m[16];
#pragma unroll
            for (int wd = 0; wd < 16; wd++) {
                uint32_t word = 0;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t k = 4 * wd + q;
                    word |= (uint32_t)(k < have ? fs->md5_buffer[k] : p[k - have]) << (8 * q);
                }
                m[wd] = word;
            }
            md5_compress(st, m);
        }
    }
    // Every lane holds the same state, which hipcc would otherwise keep in
    // SGPRs (the LDS reads are wave-uniform) and run on the scalar unit with a
    // v_readfirstlane per step; an opaque per-lane zero keeps it in VGPRs.
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
#pragma unroll
    for (int k = 0; k < 4; k++)
        st[k] ^= z;
    __syncthreads();
    for (uint64_t s = 0; s < nslots; s++) {
        const uint4 *R = ring + (s & 1) * (kChainSlotBlocks * 16);
        const uint32_t nb = (uint32_t)uniform64(nblk - s * kChainSlotBlocks < kChainSlotBlocks
                                                    ? nblk - s * kChainSlotBlocks : kChainSlotBlocks);
        uint4 ga[4], gb[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            ga[k] = R[k];
        for (uint32_t j = 0; j < nb; j++) {
            const uint4 *B = R + 16 * j;
            const uint4 *N = R + (j + 1 < nb ? 16 * (j + 1) : 0);  // the next block's first round
            uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
            // each round's sums are read while the round before is computed
#pragma unroll
            for (int k = 0; k < 4; k++)
                gb[k] = B[4 + k];
            __builtin_amdgcn_sched_barrier(0);
            md5_round_km<0>(a, b, c, d, ga);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < 4; k++)
                ga[k] = B[8 + k];
            __builtin_amdgcn_sched_barrier(0);
            md5_round_km<1>(a, b, c, d, gb);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < 4; k++)
                gb[k] = B[12 + k];
            __builtin_amdgcn_sched_barrier(0);
            md5_round_km<2>(a, b, c, d, ga);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < 4; k++)
                ga[k] = N[k];
            __builtin_amdgcn_sched_barrier(0);
            md5_round_km<3>(a, b, c, d, gb);
            __builtin_amdgcn_sched_barrier(0);
            st[0] += a;
            st[1] += b;
            st[2] += c;
            st[3] += d;
        }
        __syncthreads();
    }
    const uint8_t *tp = s0 + (nblk << 6);
    if (fs) {
        if (lane == 0) {
            // the new pending bytes: the chunk appended to a still-partial
            // buffer, or the chunk's last (L - pre) & 63 bytes
            const uint32_t r = (uint32_t)((L - pre) & 63u);
            if (have && have + L < 64) {
                for (uint32_t k = 0; k < (uint32_t)L; k++)
                    fs->md5_buffer[have + k] = p[k];
            } else {
                for (uint32_t k = 0; k < r; k++)
                    fs->md5_buffer[k] = tp[k];
            }
#pragma unroll
            for (int k = 0; k < 4; k++)
                fs->md5_state[k] = st[k];
            uint32_t cnt[2] = {fs->md5_count[0], fs->md5_count[1]};
            count_add(cnt, L);
            fs->md5_count[0] = cnt[0];
            fs->md5_count[1] = cnt[1];
        }
        return;
    }
    md5_finish(st, tp, L);
    if (lane == 0) {
        if (sig_out)  // memcpy(sig + 8, md5 digest, 16) (storage/storage_service.c:119)
            store_sig(sig_out + 24ull * f, L, st[0], st[1], st[2], st[3]);
        if (codes_out)
            reinterpret_cast<int4 *>(codes_out)[f] = make_int4((int)st[0], (int)st[1], (int)st[2], (int)st[3]);
    }
}

// The same chain on one wave with no helper (md5_chain_wave): lane i makes
// step i's sums of each 8-block slot two slots ahead into the wave's own LDS
// ring (~1 % of the chain's instructions), so four chains fit a CU, one per
// SIMD.  Used when a batch has more big files than CUs and at most one per
// SIMD; with at most one per CU the helper form above is faster (18 % on
// config 4 --method md5, profiles/r06/chain_wave_ab.txt).
constexpr uint32_t kWaveSlotBlocks = 8;  // blocks per LDS slot: 8 x 64 sums = 2 KiB

// ring: two slots, 4 KiB of LDS, this wave's own.  fs != nullptr: the
// state-carrying update (fdfs_gpu_update_batch): the chunk continues fs's
// MD5 -- the bytes my_md5_update left pending are completed first from the
// chunk's head, the chunk's last bytes become the new pending buffer, and the
// byte count advances (the CRC comes from big_patch_state_kernel).
__device__ __forceinline__ void md5_chain_wave(const uint8_t *p, uint64_t L, uint32_t f, uint4 *ring,
                                            uint8_t *sig_out, int32_t *codes_out, fdfs_gpu_file_state *fs)
{
    const int lane = threadIdx.x & 63;
    const uint32_t have = fs ? (fs->md5_count[0] >> 3) & 63u : 0u;  // bytes pending in fs's buffer
    const uint64_t pre = have ? (64 - have < L ? 64 - have : L) : 0;  // chunk bytes that complete them
    const uint8_t *s0 = p + pre;  // the stream of whole blocks
    const uint64_t nblk = (L - pre) >> 6;
    const uint64_t nslots = uniform64((nblk + kWaveSlotBlocks - 1) / kWaveSlotBlocks);
    const uint32_t kk = kMd5Kc[lane];
    const uint8_t *src = s0 + 4 * md5_msg_index(lane);
    // slot s: lane i holds m[g(i)] of its blocks (past the end the last
    // block's, never hashed; the loads are unconditional, see elf_chain_wave)
    auto load = [&](uint32_t (&v)[kWaveSlotBlocks], uint64_t s) {
        const uint64_t b0 = s * kWaveSlotBlocks;
#pragma unroll
        for (int j = 0; j < (int)kWaveSlotBlocks; j++) {
            const uint64_t blk = b0 + j < nblk ? b0 + j : nblk - 1;  // nblk > 0 whenever called
            __builtin_memcpy(&v[j], src + 64 * blk, 4);  // any alignment (unaligned memory mode)
        }
    };
    auto put = [&](const uint32_t (&v)[kWaveSlotBlocks], uint64_t s) {
        uint32_t *w = reinterpret_cast<uint32_t *>(ring + (s & 1) * (kWaveSlotBlocks * 16));
#pragma unroll
        for (int j = 0; j < (int)kWaveSlotBlocks; j++)
            w[64 * j + lane] = v[j] + kk;
    };
    __builtin_amdgcn_s_setprio(3);
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};  // my_md5_init
    if (fs) {
#pragma unroll
        for (int k = 0; k < 4; k++)
            st[k] = fs->md5_state[k];
        if (have && have + pre == 64) {  // my_md5_update's partial block: buffer || chunk head
            uint32_t m[16];
#pragma unroll
            for (int wd = 0; wd < 16; wd++) {
                uint32_t word = 0;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t k = 4 * wd + q;
                    word |= (uint32_t)(k < have ? fs->md5_buffer[k] : p[k - have]) << (8 * q);
                }
                m[wd] = word;
            }
            md5_compress(st, m);
        }
    }
    // Every lane holds the same state, which hipcc would otherwise keep in
    // SGPRs (the LDS reads are wave-uniform) and run on the scalar unit with a
    // v_readfirstlane per step; an opaque per-lane zero keeps it in VGPRs.
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
#pragma unroll
    for (int k = 0; k < 4; k++)
        st[k] ^= z;
    auto chain = [&](uint64_t s) {
        const uint4 *R = ring + (s & 1) * (kWaveSlotBlocks * 16);
        const uint32_t nb = (uint32_t)uniform64(nblk - s * kWaveSlotBlocks < kWaveSlotBlocks
                                                    ? nblk - s * kWaveSlotBlocks : kWaveSlotBlocks);
        uint4 ga[4], gb[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            ga[k] = R[k];
        for (uint32_t j = 0; j < nb; j++) {
            const uint4 *B = R + 16 * j;
            const uint4 *N = R + (j + 1 < nb ? 16 * (j + 1) : 0);  // the next block's first round
            uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
            // each round's sums are read while the round before is computed
#pragma unroll
            for (int k = 0; k < 4; k++)
                gb[k] = B[4 + k];
            __builtin_amdgcn_sched_barrier(0);
            md5_round_km<0>(a, b, c, d, ga);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < 4; k++)
                ga[k] = B[8 + k];
            __builtin_amdgcn_sched_barrier(0);
            md5_round_km<1>(a, b, c, d, gb);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < 4; k++)
                gb[k] = B[12 + k];
            __builtin_amdgcn_sched_barrier(0);
            md5_round_km<2>(a, b, c, d, ga);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < 4; k++)
                ga[k] = N[k];
            __builtin_amdgcn_sched_barrier(0);
            md5_round_km<3>(a, b, c, d, gb);
            __builtin_amdgcn_sched_barrier(0);
            st[0] += a;
            st[1] += b;
            st[2] += c;
            st[3] += d;
        }
    };
    // slot s + 1 goes into the ring and slot s + 2's loads go out before slot
    // s's chain (the ring's other slot was read by the chain before; one
    // wave's LDS operations run in order)
    uint32_t va[kWaveSlotBlocks], vb[kWaveSlotBlocks];
    if (nslots) {
        load(va, 0);
        put(va, 0);
        load(va, 1);
    }
    uint64_t s = 0;
    for (; s + 2 <= nslots; s += 2) {
        load(vb, s + 2);
        put(va, s + 1);
        chain(s);
        load(va, s + 3);
        put(vb, s + 2);
        chain(s + 1);
    }
    if (s < nslots) {
        put(va, s + 1);  // past the end: never read
        chain(s);
    }
    const uint8_t *tp = s0 + (nblk << 6);
    if (fs) {
        if (lane == 0) {
            // the new pending bytes: the chunk appended to a still-partial
            // buffer, or the chunk's last (L - pre) & 63 bytes
            const uint32_t r = (uint32_t)((L - pre) & 63u);
            if (have && have + L < 64) {
                for (uint32_t k = 0; k < (uint32_t)L; k++)
                    fs->md5_buffer[have + k] = p[k];
            } else {
                for (uint32_t k = 0; k < r; k++)
                    fs->md5_buffer[k] = tp[k];
            }
#pragma unroll
            for (int k = 0; k < 4; k++)
                fs->md5_state[k] = st[k];
            uint32_t cnt[2] = {fs->md5_count[0], fs->md5_count[1]};
            count_add(cnt, L);
            fs->md5_count[0] = cnt[0];
            fs->md5_count[1] = cnt[1];
        }
        return;
    }
    md5_finish(st, tp, L);
    if (lane == 0) {
        if (sig_out)  // memcpy(sig + 8, md5 digest, 16) (storage/storage_service.c:119)
            store_sig(sig_out + 24ull * f, L, st[0], st[1], st[2], st[3]);
        if (codes_out)
            reinterpret_cast<int4 *>(codes_out)[f] = make_int4((int)st[0], (int)st[1], (int)st[2], (int)st[3]);
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
// reads 128 contiguous bytes of 8 files (8 lanes x 16 B each), the data is
// written to LDS as one padded row per file, and each lane then hashes its
// own row.  The next round's loads are in flight while this round is hashed
// (two register sets, asm loads so hipcc cannot sink them to their use).
//
// A file's bytes may start at any address: the cooperative loads read each
// file's stream at its own (byte) offset, so the LDS rows always hold the
// stream 16-byte aligned.  gfx950 serves byte-misaligned 16-byte global loads
// (the unaligned memory mode ROCm configures; scripts/probes/unaligned_load
// checks it on the box): a misaligned file costs a second cache line per
// 128-byte piece, not a lane-serial byte loop.
//
// The file's CRC32 (CRC32_ex over the same bytes, storage/storage_dio.c:467)
// is computed by the same lane from the same LDS row: one pass over HBM for
// CRC + MD5.  Its table lookups are independent of the MD5 chain, so they
// fill the issue slots a latency-bound MD5 wave leaves empty.  The slice-by-16
// tables are shared by the workgroup's waves (waves are otherwise
// independent: no barrier after the table fill).  Exception: in a batch too
// small to fill the chip (big_plan_kernel, fdfs_sig.hip) the files >= the
// threshold *big_min leave their CRC to crc_seg_kernel, and their lanes hash
// MD5 alone (a 256 KiB chunk: 5.2 -> 3.0 ms of lane time,
// profiles/r02/chunk_sweep.txt); big_min == nullptr: every lane does both.
//
// ST (fdfs_gpu_update_batch): the lane continues a StorageFileContext-shaped
// state instead of starting one.  The (count / 8) % 64 bytes my_md5_update
// left pending are completed first from the chunk's head (lane-serial, < 64
// bytes, assembled in the lane's LDS row), the chunk's full blocks then take
// the staged path above, and its last bytes become the new pending buffer.
//
// LDS row stride CH+16 = 144 B: ds_write_b128 groups (8 lanes = one 128-byte
// row) and ds_read_b128 groups (16 lanes, rows f at quad 9f + const mod 16)
// are both conflict-free.
constexpr int kMd5Chunk = 128;
constexpr int kMd5Waves = 4;

template <bool SAR, bool ST>
__global__ __launch_bounds__(64 * kMd5Waves) void md5_stage_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint64_t *__restrict__ sizes, const uint32_t *__restrict__ order, uint32_t n,
    const DevTables *__restrict__ tabs, const uint64_t *__restrict__ big_min_p, uint32_t w1,
    uint32_t *__restrict__ queue,
    uint32_t *__restrict__ crc_out, uint8_t *__restrict__ sig_out, int32_t *__restrict__ codes_out,
    fdfs_gpu_file_state *__restrict__ states, const uint32_t *__restrict__ sidx,
    const uint32_t *__restrict__ nbig_p, uint32_t chain_wg, uint32_t chain_wave)
{
    constexpr int CH = kMd5Chunk;
    constexpr int PIECES = CH / 16;   // 16-byte pieces of one file's chunk
    constexpr int FPI = 64 / PIECES;  // files per load instruction
    constexpr int NLD = 64 / FPI;     // load instructions per round
    constexpr int STRIDE = CH + 16;   // padded LDS row per file
    constexpr int BPR = CH / 64;      // MD5 blocks per round
    static_assert(NLD == 8, "the asm waits below name 8 registers");
    __shared__ __attribute__((aligned(16))) uint32_t sD[16 * 256];  // also md5_chain_wg's ring
    __shared__ uint32_t sT[256];
    __shared__ __attribute__((aligned(16))) uint8_t sbuf[kMd5Waves][64 * STRIDE];
    lds_fill(sD, &tabs->t.D[0][0], 16 * 256);
    lds_fill(sT, tabs->t.T, 256);
    __syncthreads();
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

    const int lane = threadIdx.x & 63;
    // Waves take 64-file chunks of the size-descending order.  Without a
    // queue every wave is resident at once (a few per SIMD), so the kernel
    // ends with the SIMD that holds the most bytes: the first `w1` waves (one
    // workgroup per CU) take the largest chunks and the rest take the
    // remaining chunks smallest first, so a CU's second workgroup is a light
    // one.
    //
    // With a queue (the default) the grid is one workgroup per CU, one wave
    // per SIMD, and each wave takes the next chunk from a device counter
    // until none is left: the first chunks taken are the largest, and the
    // rest go to the waves whose chunks end first, so small files run in the
    // time the largest ones take instead of beside them (fewer files stream
    // at once while the longest chains run).
    const uint32_t nw = (n + 63) / 64;
    uint8_t *tile = sbuf[threadIdx.x >> 6];
    uint8_t *mine = tile + lane * STRIDE;
    const uint8_t *safe = reinterpret_cast<const uint8_t *>(tabs);  // >= 16 readable bytes
    const uint32_t K16 = tabs->t.K16;
    const uint64_t big_min = big_min_p ? *big_min_p : ~0ull;
    // With a queue, the first chain workgroups: with *nbig <= chain_wg big
    // files (at most one per CU) big file i runs on workgroup i
    // (md5_chain_wg, a helper wave beside it), with up to chain_wave (one per
    // SIMD) on wave i (md5_chain_wave); the waves of the queue skip them.
    uint32_t nchain = 0;
    if (queue && chain_wave) {
        const uint32_t wpb = blockDim.x >> 6;
        uint32_t cwgs = (chain_wave + wpb - 1) / wpb;
        cwgs = cwgs > chain_wg ? cwgs : chain_wg;
        const uint32_t nb = __builtin_amdgcn_readfirstlane(*nbig_p);
        nchain = nb <= chain_wave ? nb : 0;
        if (blockIdx.x < cwgs) {
            const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            if (nchain <= chain_wg) {
                if (blockIdx.x < nchain) {
                    const uint32_t fc = order[blockIdx.x];
                    if (fc < n)  // else a stale order entry (flagged by big_plan_kernel)
                        md5_chain_wg(base + offs[fc], sizes[fc], fc, wv, reinterpret_cast<uint4 *>(sD), sig_out,
                                     codes_out, ST ? states + (sidx ? sidx[fc] : fc) : nullptr);
                }
            } else {
                const uint32_t id = blockIdx.x * wpb + wv;
                if (id < nchain) {
                    const uint32_t fc = order[id];
                    if (fc < n)
                        md5_chain_wave(base + offs[fc], sizes[fc], fc,
                                       reinterpret_cast<uint4 *>(sD) + wv * (2 * kWaveSlotBlocks * 16), sig_out,
                                       codes_out, ST ? states + (sidx ? sidx[fc] : fc) : nullptr);
                }
            }
            return;
        }
    }
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
    bool valid = i < n;
    uint32_t f = valid ? order[i] : 0;
    if (f >= n) {  // a stale order entry (the binning flagged it): no file
        valid = false;
        f = 0;
    }
    if (nchain && valid && sizes[f] >= big_min)  // a chain workgroup's file
        valid = false;
    const uint64_t L = valid ? sizes[f] : 0;
    const uint8_t *p = valid ? base + offs[f] : safe;
    const bool small = L < big_min;  // else the CRC comes from crc_seg_kernel
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};  // my_md5_init
    uint32_t c = 0xFFFFFFFFu;  // CRC32_XINIT (storage/storage_service.c:7149)
    fdfs_gpu_file_state *fs = nullptr;
    uint32_t have = 0;  // bytes pending in the state's MD5 buffer
    uint64_t pre = 0;   // chunk bytes that complete them
    if constexpr (ST) {
        if (valid) {
            fs = states + (sidx ? sidx[f] : f);
            c = (uint32_t)fs->crc32;
#pragma unroll
            for (int k = 0; k < 4; k++)
                st[k] = fs->md5_state[k];
            have = (fs->md5_count[0] >> 3) & 63u;
        }
        if (have) {  // my_md5_update's partial block: buffer || chunk head
            pre = 64 - have < L ? 64 - have : L;
            for (uint32_t k = 0; k < have; k++)
                mine[k] = fs->md5_buffer[k];
            for (uint32_t k = 0; k < (uint32_t)pre; k++) {
                const uint32_t b = p[k];
                mine[have + k] = (uint8_t)b;
                if (small)
                    c = crc_byte<SAR>(sT, c, b);
            }
            if (have + pre == 64) {
                const uint4 *q = reinterpret_cast<const uint4 *>(mine);
                const uint4 a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
                const uint32_t m[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                                        a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
                md5_compress(st, m);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    const uint8_t *s0 = p + pre;  // the stream of whole blocks
    const uint64_t nblk = (L - pre) >> 6;

    auto block = [&](uint4 a0, uint4 a1, uint4 a2, uint4 a3) {
        const uint32_t m[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                                a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
        md5_compress(st, m);
        if (small) {
            c = chain16<SAR>(sD, c, a0, K16);
            c = chain16<SAR>(sD, c, a1, K16);
            c = chain16<SAR>(sD, c, a2, K16);
            c = chain16<SAR>(sD, c, a3, K16);
        }
    };

    {
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
            lp[k] = reinterpret_cast<const uint8_t *>(__shfl((uintptr_t)s0, src)) + piece * 16;
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
    }
    if (valid) {
        const uint8_t *tp = s0 + (nblk << 6);
        const uint32_t r = (uint32_t)((L - pre) & 63u);
        for (uint32_t k = 0; k < r && small; k++)  // CRC of the tail bytes
            c = crc_byte<SAR>(sT, c, tp[k]);
        if constexpr (ST) {
            // the new pending bytes: the chunk appended to a still-partial
            // buffer, or the chunk's last (L - pre) & 63 bytes
            if (have && have + L < 64) {
                for (uint32_t k = 0; k < (uint32_t)L; k++)
                    fs->md5_buffer[have + k] = p[k];
            } else {
                for (uint32_t k = 0; k < r; k++)
                    fs->md5_buffer[k] = tp[k];
            }
            if (small)  // else big_patch_state_kernel carries the segmented CRC
                fs->crc32 = (int32_t)c;
#pragma unroll
            for (int k = 0; k < 4; k++)
                fs->md5_state[k] = st[k];
            uint32_t cnt[2] = {fs->md5_count[0], fs->md5_count[1]};
            count_add(cnt, L);
            fs->md5_count[0] = cnt[0];
            fs->md5_count[1] = cnt[1];
        } else {
            md5_finish(st, tp, L);
            if (small)  // else big_patch_kernel writes the segmented CRC
                crc_out[f] = c ^ 0xFFFFFFFFu;  // CRC32_FINAL (storage/storage_dio.c:500)
            if (sig_out)  // memcpy(sig + 8, md5 digest, 16) (storage/storage_service.c:119)
                store_sig(sig_out + 24ull * f, L, st[0], st[1], st[2], st[3]);
            if (codes_out)
                reinterpret_cast<int4 *>(codes_out)[f] =
                    make_int4((int)st[0], (int)st[1], (int)st[2], (int)st[3]);
        }
    }
    if (!queue)
        break;
    uint32_t c1 = 0;
    if (lane == 0)
        c1 = atomicAdd(queue, 1u);
    chunk = __shfl(c1, 0);
    }
}

// ------------------------------------------------ MD5 path, paired waves
//
// The one-shot batch form (no state) of the kernel above with the CRC taken
// off the MD5 lane.  A workgroup is two waves on one 64-file chunk at a time:
// wave 0 runs the 64 MD5 chains only; wave 1 issues the cooperative loads,
// stages each round's 128 bytes of every file in LDS and computes the CRCs
// from the same rows.  In the fused form the CRC's ~35 instructions per 16
// bytes sit on the MD5 lane, whose wave issues one instruction every several
// cycles (a dependent chain at one wave per SIMD): the largest file's chain
// was 80 ms fused against 53-58 ms for MD5 alone (profiles/r02).  Here the
// CRC runs on a second wave that fills the issue slots the MD5 chain leaves
// empty, and the MD5 wave has neither loads nor LDS stores to issue.
//
// Rows are double-buffered: the loader writes round r into buffer r & 1,
// both waves meet at one barrier per round, then hash that buffer.  The
// loader writes buffer (r + 1) & 1 only after the barrier of round r, which
// the MD5 wave reaches only once it has finished round r - 1 on that buffer.
// The barrier is s_barrier after lgkmcnt(0) alone: the loader's next round of
// loads stays in flight across it (__syncthreads would wait for them).
// Four workgroups per CU (35.8 KB of LDS each), the same 64 MD5 lanes per
// SIMD as the fused form's one wave per SIMD.
// Issue priority from a wave-uniform count of remaining 128-byte rounds:
// the waves with the most work left
// issue first on their SIMDs -- longest-remaining-first, the LPT rule applied
// to the SIMD's issue arbiter -- against the hardware's oldest-wave-first
// default, which favours the workgroups dispatched first whatever they have
// left.  Every SIMD holds an MD5 wave and a loader wave of two different
// chunks, so a chunk with 3 MiB to go outranks one about to end.
// Config 3: 80.0 / 80.6 against 83.4 / 83.0 ms, alternating on one box
// (profiles/r04/probes_r04b.txt, c3_p7 against c3_p1).  Re-evaluated every
// 256 rounds (32 KiB per file), in 1 MiB units.
template <int SH = 13>
__device__ __forceinline__ void prio_by_remaining(uint64_t rem)
{
    const uint32_t q = __builtin_amdgcn_readfirstlane((uint32_t)(rem >> SH));  // 8K-round units (SH 13)
    if (q >= 3)
        __builtin_amdgcn_s_setprio(3);
    else if (q == 2)
        __builtin_amdgcn_s_setprio(2);
    else if (q == 1)
        __builtin_amdgcn_s_setprio(1);
    else
        __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ void pair_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <bool SAR>
__global__ __launch_bounds__(128) void md5_pair_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint64_t *__restrict__ sizes, const uint32_t *__restrict__ order, uint32_t n,
    const DevTables *__restrict__ tabs, const uint64_t *__restrict__ big_min_p, uint32_t *__restrict__ queue,
    uint32_t *__restrict__ crc_out, uint8_t *__restrict__ sig_out, int32_t *__restrict__ codes_out,
    const uint32_t *__restrict__ nbig_p, uint32_t chain_wg, uint32_t chain_wave)
{
    constexpr int CH = kMd5Chunk;
    constexpr int PIECES = CH / 16;
    constexpr int FPI = 64 / PIECES;
    constexpr int NLD = 64 / FPI;
    constexpr int STRIDE = CH + 16;
    constexpr int BPR = CH / 64;
    static_assert(NLD == 8, "the asm waits below name 8 registers");
    __shared__ __attribute__((aligned(16))) uint32_t sD[16 * 256];  // also md5_chain_wg's ring
    __shared__ uint32_t sT[256];
    __shared__ __attribute__((aligned(16))) uint8_t sbuf[2][64 * STRIDE];
    __shared__ uint32_t s_chunk;
    lds_fill(sD, &tabs->t.D[0][0], 16 * 256);
    lds_fill(sT, tabs->t.T, 256);
    __syncthreads();
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    // wave-uniform role (an SGPR, so both roles' barriers are scalar branches)
    const bool loader = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) != 0;
    const int lane = threadIdx.x & 63;
    const uint32_t nw = (n + 63) / 64;
    const uint8_t *safe = reinterpret_cast<const uint8_t *>(tabs);
    const uint32_t K16 = tabs->t.K16;
    const uint64_t big_min = big_min_p ? *big_min_p : ~0ull;
    // Big files (the first *nbig of the order): with *nbig <= chain_wg (at
    // most one per CU) big file i runs on workgroup i (md5_chain_wg, the
    // loader wave its helper), with up to chain_wave (one per SIMD) on wave i
    // (md5_chain_wave); the tables' LDS is the rings, and the pairs skip
    // those files.
    uint32_t nchain = 0;
    if (chain_wave && nbig_p) {
        uint32_t cwgs = (chain_wave + 1) / 2;
        cwgs = cwgs > chain_wg ? cwgs : chain_wg;
        const uint32_t nb = __builtin_amdgcn_readfirstlane(*nbig_p);
        nchain = nb <= chain_wave ? nb : 0;
        if (blockIdx.x < cwgs) {
            const uint32_t wv = loader ? 1u : 0u;
            if (nchain <= chain_wg) {
                if (blockIdx.x < nchain) {
                    const uint32_t fc = order[blockIdx.x];
                    if (fc < n)  // else a stale order entry (flagged by big_plan_kernel)
                        md5_chain_wg(base + offs[fc], sizes[fc], fc, (int)wv, reinterpret_cast<uint4 *>(sD),
                                     sig_out, codes_out, nullptr);
                }
            } else {
                const uint32_t id = blockIdx.x * 2 + wv;
                if (id < nchain) {
                    const uint32_t fc = order[id];
                    if (fc < n)
                        md5_chain_wave(base + offs[fc], sizes[fc], fc,
                                       reinterpret_cast<uint4 *>(sD) + wv * (2 * kWaveSlotBlocks * 16), sig_out,
                                       codes_out, nullptr);
                }
            }
            return;
        }
    }
    for (;;) {
        if (threadIdx.x == 64)
            s_chunk = atomicAdd(queue, 1u);
        __syncthreads();
        const uint32_t chunk = __builtin_amdgcn_readfirstlane(s_chunk);
        __syncthreads();  // s_chunk read by both waves before the next chunk's write
        if (chunk >= nw)
            break;
        const uint32_t i = chunk * 64 + lane;
        bool valid = i < n;
        uint32_t f = valid ? order[i] : 0;
        if (f >= n) {  // a stale order entry (the binning flagged it): no file
            valid = false;
            f = 0;
        }
        if (nchain && valid && sizes[f] >= big_min)  // a chain workgroup's file
            valid = false;
        const uint64_t L = valid ? sizes[f] : 0;
        const uint8_t *p = valid ? base + offs[f] : safe;
        const uint64_t nblk = L >> 6;
        uint64_t mx = nblk;
#pragma unroll
        for (int o = 32; o; o >>= 1) {
            const uint64_t y = __shfl_xor(mx, o);
            mx = y > mx ? y : mx;
        }
        const uint64_t rounds = uniform64((mx + BPR - 1) / BPR);  // SGPRs: scalar round loops
        const uint8_t *tp = p + (nblk << 6);
        if (loader) {
            const bool small = L < big_min;  // else the CRC comes from crc_seg_kernel
            const int piece = lane % PIECES, fsub = lane / PIECES;
            const uint8_t *lp[NLD];
            uint64_t lim[NLD];
#pragma unroll
            for (int k = 0; k < NLD; k++) {
                const int src = k * FPI + fsub;
                lp[k] = reinterpret_cast<const uint8_t *>(__shfl((uintptr_t)p, src)) + piece * 16;
                lim[k] = __shfl(nblk, src) * 4;
            }
            // Three register sets: round r + 2's loads are issued while round
            // r is staged and hashed (two rounds of lookahead: under the
            // batch's 3.6 TB/s a load takes longer than one round).
            u32x4 RA[NLD], RB[NLD], RC[NLD];
            auto issue = [&](u32x4 (&R)[NLD], uint64_t r) {
                const uint64_t rp = r * PIECES + piece;
#pragma unroll
                for (int k = 0; k < NLD; k++) {
                    const uint8_t *a = (rp < lim[k]) ? lp[k] + r * CH : safe;
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(R[k]) : "v"(a) : "memory");
                }
            };
            // R is the oldest of the three sets in flight.  The wait is taken
            // on every path through the loop body (only the staging is
            // conditional), so no path reaches the next issue into R's
            // registers with R's loads still in flight (tests/test_isa.py).
            auto wait_older = [&](u32x4 (&R)[NLD]) {
                asm volatile("s_waitcnt vmcnt(16)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]) :: "memory");
                asm volatile("" : "+v"(R[4]), "+v"(R[5]), "+v"(R[6]), "+v"(R[7]));
            };
            auto stage = [&](u32x4 (&R)[NLD], uint8_t *tile) {
#pragma unroll
                for (int k = 0; k < NLD; k++)
                    *reinterpret_cast<u32x4 *>(tile + (k * FPI + fsub) * STRIDE + piece * 16) = R[k];
            };
            uint32_t c = 0xFFFFFFFFu;  // CRC32_XINIT (storage/storage_service.c:7149)
            // The CRC of the whole blocks: the lane fold (fdfs_device.hpp) in
            // 32 registers, one round's 32 dwords; XINIT enters as the first
            // block's first dword (fdfs_tables.hpp Y4).
            static_assert(CH == 128, "a round is the fold's 32 dwords");
            uint32_t ring[32];
#pragma unroll
            for (int k = 0; k < 32; k++)
                ring[k] = 0;
            uint32_t zin = c ^ ((SAR && (int32_t)c < 0) ? tabs->t.Y4 : 0u);
            auto crc_round = [&](uint64_t r, const uint8_t *tile) {
                const uint4 *q = reinterpret_cast<const uint4 *>(tile + lane * STRIDE);
#pragma unroll
                for (int b = 0; b < BPR; b++)
                    if (small && r * BPR + b < nblk) {
#pragma unroll
                        for (int k = 0; k < 4; k++) {
                            const uint4 w = q[4 * b + k];
                            const int s0 = 16 * b + 4 * k;
                            ring[s0 + 0] = lane_fold_dw<SAR>(ring, s0 + 0, (b == 0 && k == 0) ? w.x ^ zin : w.x);
                            ring[s0 + 1] = lane_fold_dw<SAR>(ring, s0 + 1, w.y);
                            ring[s0 + 2] = lane_fold_dw<SAR>(ring, s0 + 2, w.z);
                            ring[s0 + 3] = lane_fold_dw<SAR>(ring, s0 + 3, w.w);
                        }
                    }
                zin = 0;  // taken by round 0
            };
            // round r's rows go to sbuf[r & 1] (the MD5 wave reads them there)
            auto round = [&](u32x4 (&R)[NLD], uint64_t r) {
                uint8_t *tile = sbuf[r & 1];
                stage(R, tile);
                pair_barrier();
                crc_round(r, tile);
            };
            issue(RA, 0);
            issue(RB, 1);
            for (uint64_t r = 0; r < rounds; r += 3) {
                if ((r & 255) < 3)  // every 256 rounds
                    prio_by_remaining(rounds - r);
                issue(RC, r + 2);
                wait_older(RA);
                round(RA, r);
                issue(RA, r + 3);
                wait_older(RB);
                if (r + 1 < rounds)
                    round(RB, r + 1);
                issue(RB, r + 4);
                wait_older(RC);
                if (r + 2 < rounds)
                    round(RC, r + 2);
            }
            // the last (past-the-end) sets
            asm volatile("s_waitcnt vmcnt(0)"
                         : "+v"(RA[0]), "+v"(RA[1]), "+v"(RA[2]), "+v"(RA[3]), "+v"(RA[4]), "+v"(RA[5]),
                           "+v"(RA[6]), "+v"(RA[7]) :: "memory");
            asm volatile("" : "+v"(RB[0]), "+v"(RB[1]), "+v"(RB[2]), "+v"(RB[3]), "+v"(RB[4]), "+v"(RB[5]),
                         "+v"(RB[6]), "+v"(RB[7]) :: "memory");
            if (valid && small) {
                if (nblk > 0) {
                    // the last 32 dwords in position order: an odd block
                    // count ends mid-ring (slot 15)
                    const bool odd = nblk & 1;
#pragma unroll
                    for (int k = 0; k < 16; k++) {
                        const uint32_t lo = ring[k], hi = ring[k + 16];
                        ring[k] = odd ? hi : lo;
                        ring[k + 16] = odd ? lo : hi;
                    }
                    c = lane_fold_finish<SAR>(sD, K16, ring);
                }
                const uint32_t rt = (uint32_t)(L & 63u);
                for (uint32_t k = 0; k < rt; k++)  // CRC of the tail bytes
                    c = crc_byte<SAR>(sT, c, tp[k]);
                crc_out[f] = c ^ 0xFFFFFFFFu;  // CRC32_FINAL (storage/storage_dio.c:500)
            }
        } else {
            uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};  // my_md5_init
            const uint8_t *mine = &sbuf[0][0] + lane * STRIDE;
            for (uint64_t r = 0; r < rounds; r++) {
                if ((r & 255) == 0)
                    prio_by_remaining(rounds - r);
                pair_barrier();
                const uint4 *q = reinterpret_cast<const uint4 *>(mine + (r & 1) * (64 * STRIDE));
                // block b + 1's words are read from LDS (for every lane,
                // outside the per-lane branch) while block b is compressed
                uint4 cur[4] = {q[0], q[1], q[2], q[3]};
#pragma unroll
                for (int b = 0; b < BPR; b++) {
                    uint4 nxt[4];
                    if (b + 1 < BPR) {
#pragma unroll
                        for (int k = 0; k < 4; k++)
                            nxt[k] = q[4 * (b + 1) + k];
                    }
                    if (r * BPR + b < nblk) {
                        const uint32_t m[16] = {cur[0].x, cur[0].y, cur[0].z, cur[0].w, cur[1].x, cur[1].y,
                                                cur[1].z, cur[1].w, cur[2].x, cur[2].y, cur[2].z, cur[2].w,
                                                cur[3].x, cur[3].y, cur[3].z, cur[3].w};
                        md5_compress(st, m);
                    }
                    if (b + 1 < BPR) {
#pragma unroll
                        for (int k = 0; k < 4; k++)
                            cur[k] = nxt[k];
                    }
                }
            }
            if (valid) {
                md5_finish(st, tp, L);
                if (sig_out)  // memcpy(sig + 8, md5 digest, 16) (storage/storage_service.c:119)
                    store_sig(sig_out + 24ull * f, L, st[0], st[1], st[2], st[3]);
                if (codes_out)
                    reinterpret_cast<int4 *>(codes_out)[f] =
                        make_int4((int)st[0], (int)st[1], (int)st[2], (int)st[3]);
            }
        }
    }
}

hipError_t launch_md5_stage(bool sar, const uint8_t *base, const uint64_t *offs,
                            const uint64_t *sizes, uint32_t n, const uint32_t *order,
                            const DevTables *tabs, const uint64_t *big_min, uint32_t *queue, uint32_t *crc_out,
                            uint8_t *sig_out, int32_t *codes_out, fdfs_gpu_file_state *states,
                            const uint32_t *sidx, unsigned ncu, hipStream_t st,
                            const uint32_t *nbig, uint32_t chain_cap)
{
    if (ncu == 0)
        return hipErrorInvalidValue;
    constexpr unsigned kBlk = 64 * kMd5Waves;
    const uint32_t nw = (n + 63) / 64;
    if (queue && !states) {  // one-shot batches: the wave pairs (queue zeroed by the caller)
        const unsigned g = 4u * ncu;
        // the chain workgroups (one per big file up to one per CU, or a
        // wave per big file up to one per SIMD), then the pairs' grid
        if (!nbig || !big_min)
            chain_cap = 0;
        const uint32_t wv_cap = n < chain_cap ? n : chain_cap;
        const uint32_t wg_cap = wv_cap < chain_cap / 4 ? wv_cap : chain_cap / 4;
        const uint32_t cw = (wv_cap + 1) / 2;
        const unsigned grid2 = (cw > wg_cap ? cw : wg_cap) + (g < nw ? g : nw);
        if (sar)
            md5_pair_kernel<true><<<grid2, 128, 0, st>>>(base, offs, sizes, order, n, tabs, big_min, queue, crc_out,
                                                         sig_out, codes_out, nbig, wg_cap, wv_cap);
        else
            md5_pair_kernel<false><<<grid2, 128, 0, st>>>(base, offs, sizes, order, n, tabs, big_min, queue, crc_out,
                                                          sig_out, codes_out, nbig, wg_cap, wv_cap);
        return hipGetLastError();
    }
    unsigned grid = (n + kBlk - 1) / kBlk;
    uint32_t wv_cap = 0, wg_cap = 0;
    if (queue) {  // queue zeroed by the caller (launch_sig_lane's workspace memset)
        grid = ncu < (nw + kMd5Waves - 1) / kMd5Waves ? ncu : (nw + kMd5Waves - 1) / kMd5Waves;
        if (nbig && big_min) {  // the chain workgroups first
            wv_cap = n < chain_cap ? n : chain_cap;
            wg_cap = wv_cap < chain_cap / 4 ? wv_cap : chain_cap / 4;
        }
        const uint32_t cw = (wv_cap + kMd5Waves - 1) / kMd5Waves;
        grid += cw > wg_cap ? cw : wg_cap;
    }
    const uint32_t w1 = ncu * kMd5Waves;
#define MD5_LAUNCH(S, T)                                                                                  \
    md5_stage_kernel<S, T><<<grid, kBlk, 0, st>>>(base, offs, sizes, order, n, tabs, big_min, w1, queue, \
                                                  crc_out, sig_out, codes_out, states, sidx, nbig, wg_cap, wv_cap)
    if (states)
        sar ? MD5_LAUNCH(true, true) : MD5_LAUNCH(false, true);
    else
        sar ? MD5_LAUNCH(true, false) : MD5_LAUNCH(false, false);
#undef MD5_LAUNCH
    return hipGetLastError();
}

}  // namespace fdfs

