// Chunked (state-carrying) form of the upload path: the per-file
// StorageFileContext state (storage/storage_nio.h:94-96) that
// storage_write_to_file initialises (storage/storage_service.c:7147-7161),
// dio_write_file advances one received chunk at a time
// (storage/storage_dio.c:465-483) and finalises after the last chunk
// (storage/storage_dio.c:498-515), for a batch of uploads per call.
//
// The heavy per-chunk work is the one-shot kernels run in their state mode
// (sig_hash_kernel / md5_stage_kernel, fdfs_hash.hip / fdfs_md5.hip) or, for
// CRC only, the segmented kernel followed by crc_carry_kernel below.  This
// file holds the small per-file kernels around them.
#include "fdfs_device.hpp"
#include "fdfs_kernels.hpp"
#include "fdfs_md5.hpp"

namespace fdfs {

static_assert(sizeof(fdfs_gpu_file_state) == 128, "fdfs_gpu_file_state is 128 bytes");

__global__ void state_init_kernel(fdfs_gpu_file_state *__restrict__ states, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    fdfs_gpu_file_state *fs = states + i;
    fs->crc32 = (int32_t)0xFFFFFFFFu;  // CRC32_XINIT (storage/storage_service.c:7149)
    fs->hash_codes[0] = (int32_t)0xFFFFFFFFu;  // INIT_HASH_CODES4 (:7156)
    fs->hash_codes[1] = 0;
    fs->hash_codes[2] = 0;
    fs->hash_codes[3] = 0;
    fs->md5_state[0] = 0x67452301u;  // my_md5_init (:7160)
    fs->md5_state[1] = 0xefcdab89u;
    fs->md5_state[2] = 0x98badcfeu;
    fs->md5_state[3] = 0x10325476u;
    fs->md5_count[0] = 0;
    fs->md5_count[1] = 0;
}

// CRC_ONLY update: crc[f] = CRC32_FINAL(CRC32_ex(chunk f, XINIT)) as the
// segmented kernel leaves it; the chunk's own running value X carries over
// as CRC32_ex(d, X) = crc ^ ~0 ^ M^|d| (X ^ ~0) (linear over GF(2)).
__global__ void crc_carry_kernel(const uint32_t *__restrict__ crc, const uint64_t *__restrict__ sizes,
                                 uint32_t n, const uint32_t *__restrict__ sidx,
                                 fdfs_gpu_file_state *__restrict__ states, const DevTables *__restrict__ tabs)
{
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n)
        return;
    const uint64_t L = sizes[f];
    fdfs_gpu_file_state *fs = states + (sidx ? sidx[f] : f);
    fs->crc32 = (int32_t)(crc[f] ^ 0xFFFFFFFFu ^ advance_bytes(tabs->t, ~(uint32_t)fs->crc32, L));
    uint32_t cnt[2] = {fs->md5_count[0], fs->md5_count[1]};
    count_add(cnt, L);
    fs->md5_count[0] = cnt[0];
    fs->md5_count[1] = cnt[1];
}

// CRC32_FINAL, FINISH_HASH_CODES4 / my_md5_final and
// STORAGE_GEN_FILE_SIGNATURE (storage/storage_service.c:106-120) of state
// sidx[i]; the state itself is left as it is.
__global__ void final_kernel(int method, const fdfs_gpu_file_state *__restrict__ states,
                             const uint32_t *__restrict__ sidx, uint32_t n, uint32_t *__restrict__ crc_out,
                             uint8_t *__restrict__ sig_out, int32_t *__restrict__ codes_out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const fdfs_gpu_file_state *fs = states + (sidx ? sidx[i] : i);
    const uint32_t crc = (uint32_t)fs->crc32 ^ 0xFFFFFFFFu;  // CRC32_FINAL (storage/storage_dio.c:500)
    crc_out[i] = crc;
    if (method == FDFS_SIG_CRC_ONLY)
        return;
    const uint32_t lo = fs->md5_count[0], hi = fs->md5_count[1];
    const uint64_t L = ((uint64_t)hi << 32 | lo) >> 3;
    uint32_t w[4];
    if (method == FDFS_SIG_HASH) {  // FINISH_HASH_CODES4 (:508): only h[0] is finalised
        w[0] = (uint32_t)fs->hash_codes[0] ^ 0xFFFFFFFFu;
        w[1] = (uint32_t)fs->hash_codes[1];
        w[2] = (uint32_t)fs->hash_codes[2];
        w[3] = (uint32_t)fs->hash_codes[3];
    } else {  // my_md5_final (:512) over the pending (count / 8) % 64 bytes
        uint32_t st[4] = {fs->md5_state[0], fs->md5_state[1], fs->md5_state[2], fs->md5_state[3]};
        uint32_t m[16];
        const uint32_t *b = reinterpret_cast<const uint32_t *>(fs->md5_buffer);
#pragma unroll
        for (int k = 0; k < 16; k++)
            m[k] = b[k];
        md5_pad_compress(st, m, (lo >> 3) & 63u, lo, hi);
#pragma unroll
        for (int k = 0; k < 4; k++)
            w[k] = st[k];
    }
    if (codes_out)
        reinterpret_cast<int4 *>(codes_out)[i] = make_int4((int)w[0], (int)w[1], (int)w[2], (int)w[3]);
    if (sig_out) {  // long2buff(size), then int2buff x4 (hash) or the raw digest (MD5)
        uint32_t *sp = reinterpret_cast<uint32_t *>(sig_out + 24ull * i);
        sp[0] = bswap32((uint32_t)(L >> 32));
        sp[1] = bswap32((uint32_t)L);
#pragma unroll
        for (int k = 0; k < 4; k++)
            sp[2 + k] = method == FDFS_SIG_HASH ? bswap32(w[k]) : w[k];
    }
}

__global__ void crc_combine_kernel(const uint32_t *__restrict__ a, const uint32_t *__restrict__ b,
                                   const uint64_t *__restrict__ len_b, uint32_t n, uint32_t *__restrict__ out,
                                   const DevTables *__restrict__ tabs)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        out[i] = advance_bytes(tabs->t, a[i], len_b[i]) ^ b[i];
}

static unsigned blocks(uint32_t n) { return (n + 255) / 256; }

// fdfs_gpu_update_batch's contract check: a state index may appear at most
// once per call (two chunks on one state would race).  Open addressing on
// `size` (a power of two >= 2n) u32 slots, pre-filled with ~0: a claim that
// meets its own value is a duplicate.  flag |= 1 on a duplicate, 2 on the
// reserved value ~0.
__global__ void sidx_fill_kernel(uint32_t *__restrict__ table, uint32_t size)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < size; i += gridDim.x * blockDim.x)
        table[i] = ~0u;
}

__global__ void sidx_dup_kernel(const uint32_t *__restrict__ sidx, uint32_t n, uint32_t *__restrict__ table,
                                uint32_t size, uint32_t *__restrict__ flag)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t v = sidx[i];
    if (v == ~0u) {
        atomicOr(flag, 2u);
        return;
    }
    for (uint32_t h = (v * 0x9E3779B1u) & (size - 1);; h = (h + 1) & (size - 1)) {
        const uint32_t cur = atomicCAS(&table[h], ~0u, v);
        if (cur == ~0u)
            return;
        if (cur == v) {
            atomicOr(flag, 1u);
            return;
        }
    }
}

uint32_t sidx_table_size(uint32_t n)
{
    uint32_t s = 64;
    while (s < 2ull * n && s < (1u << 31))
        s <<= 1;
    return s;
}

hipError_t launch_sidx_check(const uint32_t *sidx, uint32_t n, uint32_t *table, uint32_t *flag, hipStream_t st)
{
    const uint32_t size = sidx_table_size(n);
    const uint32_t g = (size + 255) / 256;
    sidx_fill_kernel<<<g < 4096 ? g : 4096, 256, 0, st>>>(table, size);
    hipError_t e = launch_zero_u32(flag, 1, st);
    if (e != hipSuccess)
        return e;
    sidx_dup_kernel<<<blocks(n), 256, 0, st>>>(sidx, n, table, size, flag);
    return hipGetLastError();
}

hipError_t launch_state_init(fdfs_gpu_file_state *states, uint32_t n, hipStream_t st)
{
    state_init_kernel<<<blocks(n), 256, 0, st>>>(states, n);
    return hipGetLastError();
}

hipError_t launch_crc_carry(const uint32_t *crc, const uint64_t *sizes, uint32_t n, const uint32_t *sidx,
                            fdfs_gpu_file_state *states, const DevTables *tabs, hipStream_t st)
{
    crc_carry_kernel<<<blocks(n), 256, 0, st>>>(crc, sizes, n, sidx, states, tabs);
    return hipGetLastError();
}

// Split-file CRC (fdfs_gpu_crc_batch_global).  Piece i holds bytes
// [start, start + len) of file f, and crc[i] = CRC32_FINAL(CRC32_ex(piece,
// XINIT)) from crc_seg_kernel.  Over GF(2) the file's register is
//   CRC32_ex(file, XINIT) = M^size XINIT ^ XOR_i M^(size - start_i - len_i) CRC32_ex(piece_i, 0)
// whenever the pieces tile the file, in any order and on any rank, and
// CRC32_ex(piece, 0) = ~crc[i] ^ M^len XINIT.  A rank's block (CrcParts)
// holds per file the XOR of its pieces' terms, the sum of their lengths and
// the sum of H(end) - H(start) over them (H a 64-bit mix of a position, sums
// mod 2^64), and an error word (bit 0: a piece names a file >= nfiles or runs
// past its file's end; such a piece is dropped).
//
// Why the boundary sum: the number of pieces covering byte x is (starts <=
// x) - (ends <= x), so it is 1 on [0, size) and 0 elsewhere -- every byte
// covered exactly once -- if and only if the multiset of ends minus the
// multiset of starts is {size} - {0}.  Summing H over that difference checks
// this with a 2^-64-class false-accept chance (overlapping pieces plus a
// matching gap, e.g. [0, 10) twice for a 20-byte file, pass the length sum
// alone; they fail here).
__device__ __forceinline__ uint64_t piece_pos_hash(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void crc_piece_kernel(const uint32_t *__restrict__ crc, const uint64_t *__restrict__ pfile,
                                 const uint64_t *__restrict__ pstart, const uint64_t *__restrict__ plen,
                                 uint32_t np, const uint64_t *__restrict__ fsize, uint64_t nfiles,
                                 CrcParts blk, const DevTables *__restrict__ tabs)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np)
        return;
    const uint64_t f = pfile[i], a = pstart[i], len = plen[i];
    if (f >= nfiles) {
        atomicOr(blk.err(0), 1u);
        return;
    }
    const uint64_t size = fsize[f];
    if (a > size || len > size - a) {
        atomicOr(blk.err(0), 1u);
        return;
    }
    const uint32_t c0 = ~crc[i] ^ advance_bytes(tabs->t, 0xFFFFFFFFu, len);
    atomicXor(blk.word(0, f), advance_bytes(tabs->t, c0, size - a - len));
    atomicAdd(reinterpret_cast<unsigned long long *>(blk.len(0, f)), (unsigned long long)len);
    atomicAdd(reinterpret_cast<unsigned long long *>(blk.bnd(0, f)),
              (unsigned long long)(piece_pos_hash(a + len) - piece_pos_hash(a)));
}

// The fold over the ranks' blocks: crc_out[f] = CRC32_FINAL(M^size XINIT ^
// XOR_r term_r[f]); err_out[0] = the mask of ranks whose error word is set,
// err_out[1] = the files whose pieces do not tile them exactly: lengths that
// do not add up to the size, or a boundary sum other than H(size) - H(0)
// (zeroed by the caller).
__global__ void crc_fold_kernel(CrcParts blk, uint32_t nranks, const uint64_t *__restrict__ fsize, uint64_t nfiles,
                                uint32_t *__restrict__ crc_out, uint64_t *__restrict__ err_out,
                                const DevTables *__restrict__ tabs)
{
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        uint64_t m = 0;
        for (uint32_t r = 0; r < nranks; r++)
            if (*blk.err(r))
                m |= 1ull << r;
        err_out[0] = m;
    }
    uint32_t bad = 0;
    for (uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; f < nfiles;
         f += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t size = fsize[f];
        uint32_t x = advance_bytes(tabs->t, 0xFFFFFFFFu, size);
        uint64_t covered = 0, bsum = 0;
        for (uint32_t r = 0; r < nranks; r++) {
            x ^= *blk.word(r, f);
            covered += *blk.len(r, f);
            bsum += *blk.bnd(r, f);
        }
        crc_out[f] = ~x;
        bad += covered != size || bsum != piece_pos_hash(size) - piece_pos_hash(0);
    }
    if (bad)
        atomicAdd(reinterpret_cast<unsigned long long *>(err_out + 1), (unsigned long long)bad);
}

hipError_t launch_crc_pieces(const uint32_t *crc, const uint64_t *pfile, const uint64_t *pstart, const uint64_t *plen,
                             uint32_t np, const uint64_t *fsize, uint64_t nfiles, const CrcParts &blk,
                             const DevTables *tabs, hipStream_t st)
{
    if (np)
        crc_piece_kernel<<<blocks(np), 256, 0, st>>>(crc, pfile, pstart, plen, np, fsize, nfiles, blk, tabs);
    return hipGetLastError();
}

hipError_t launch_crc_fold(const CrcParts &blk, uint32_t nranks, const uint64_t *fsize, uint64_t nfiles,
                           uint32_t *crc_out, uint64_t *err_out, const DevTables *tabs, hipStream_t st)
{
    const uint64_t g = (nfiles + 255) / 256;
    crc_fold_kernel<<<(unsigned)(g < 1 ? 1 : g > 16384 ? 16384 : g), 256, 0, st>>>(blk, nranks, fsize, nfiles, crc_out,
                                                                                err_out, tabs);
    return hipGetLastError();
}

hipError_t launch_final(int method, const fdfs_gpu_file_state *states, const uint32_t *sidx, uint32_t n,
                        uint32_t *crc_out, uint8_t *sig_out, int32_t *codes_out, hipStream_t st)
{
    final_kernel<<<blocks(n), 256, 0, st>>>(method, states, sidx, n, crc_out, sig_out, codes_out);
    return hipGetLastError();
}

hipError_t launch_crc_combine(const uint32_t *a, const uint32_t *b, const uint64_t *len_b, uint32_t n,
                              uint32_t *out, const DevTables *tabs, hipStream_t st)
{
    crc_combine_kernel<<<blocks(n), 256, 0, st>>>(a, b, len_b, n, out, tabs);
    return hipGetLastError();
}

}  // namespace fdfs
