// Launcher declarations shared between the kernel TUs and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../../include/fdfs_gpu.h"
#include "fdfs_tables.hpp"

namespace fdfs {

struct DevTables;

constexpr int kSegBlock = 512;             // threads per crc_seg_kernel / crc_tab_kernel workgroup
constexpr int kSizeBins = 2048;            // size bins of the lane-path counting sort
constexpr int kLaneWsDwords = 2 * kSizeBins + 64;  // size-bin histogram + cursors + MD5 chunk queue + error word
// Lane-path error word (zeroed with the histogram at every launch): bit 0 =
// the size binning placed a file outside [0, n) or read a file index >= n
// (a histogram that was not zero before counting); such files are skipped,
// never read or written out of bounds.  The API copies it to the host after
// the launch and fails the context's next call with EIO (through a
// per-context error count that only grows, fdfs_api.cpp lane_err_note).
constexpr int kLaneErrWord = 2 * kSizeBins + 32;

// signature path (fdfs_sig.hip)
uint64_t scan_workspace_elems(uint64_t n);
// Zero n dwords on st with a kernel (ordered like any kernel node when the
// sequence is captured in a hipGraph; see zero_u32_kernel).
hipError_t launch_zero_u32(void *p, uint64_t ndwords, hipStream_t st);
// count += 1 if *word != 0 (word == nullptr: unconditionally), one thread.
hipError_t launch_lane_err_count(const uint32_t *word, uint64_t *count, uint64_t *slot, hipStream_t st);
hipError_t launch_exclusive_scan(const uint64_t *in, uint64_t n, uint64_t *out, uint64_t *bsum,
                                 hipStream_t st);
// Lane paths: files of at least a threshold T get their CRC (and for HASH
// simple_hash and Time33) from segment-parallel kernels; their lanes keep
// only ELFHash (HASH, a wave of such files is issue-bound, see
// fdfs_hash.hip) or MD5.  Batches of more than lat_files files (one wave per
// SIMD) use T = kBigCrcMin (HASH) or no offload (MD5: its single fused pass
// is HBM-bound there); smaller ones are latency-bound and big_plan_kernel
// picks T from the size histogram (fdfs_sig.hip).
constexpr uint64_t kBigCrcMin = 4ull << 20;
struct BigCrcWs {  // device arrays of n entries (seg_first n + 1)
    uint32_t *nbig;
    uint64_t *offs, *sizes, *seg_first;
    uint32_t *crc;
    uint32_t *poly;      // [2n]: simple_hash, Time33 per big file
    uint64_t *big_min;   // [1]: the T big_plan_kernel chose (read by the lane kernel)
    uint32_t lat_files;  // host: batches up to this many files choose T adaptively (0: never)
    uint32_t ncu = 0;    // host: the context device's CU count (fdfs_gpu_open), sizes persistent grids
};
hipError_t launch_poly_seg(const uint8_t *base, const uint64_t *boffs, const uint64_t *bsizes,
                           const uint64_t *seg_first, const uint32_t *nbig, uint32_t *bpoly,
                           unsigned grid, hipStream_t st);
// Lane-per-file paths (HASH / MD5).  states == nullptr: one-shot over whole
// files (outputs crc_out / sig_out / codes_out).  states != nullptr: the
// chunked update (fdfs_gpu_update_batch): chunk f continues and rewrites
// states[sidx ? sidx[f] : f], and no output is written.
hipError_t launch_sig_lane(bool sar, int method, const uint8_t *base, const uint64_t *offs,
                           const uint64_t *sizes, uint32_t n, uint32_t *hist, uint32_t *order,
                           const BigCrcWs *big, const DevTables *tabs, uint32_t *crc_out,
                           uint8_t *sig_out, int32_t *codes_out, fdfs_gpu_file_state *states,
                           const uint32_t *sidx, unsigned ncu, hipStream_t st,
                           hipEvent_t ev0, hipEvent_t ev1);
// The CRC of n files, CRC only: the files below kFoldMinBytes through
// crc_tab_kernel, the others through crc_seg_kernel (the sparse fold), each
// over its own segment list.  Workspace: nseg[2 n], seg_first[2 (n + 1)],
// bsum[2 scan_workspace_elems(n)] (crc_plan_elems).
// (the measured crossover: 64 KiB files 0.92 ms per 4 GiB on the fold
// against 0.80 on the table kernel, 128 KiB files 0.69-0.71 against 0.78;
// profiles/r05/crc_size_sweep.txt)
constexpr uint64_t kFoldMinBytes = 96 * 1024;
hipError_t launch_crc_seg(bool sar, const uint8_t *base, const uint64_t *offs, const uint64_t *sizes,
                          uint32_t n, uint64_t *nseg, uint64_t *seg_first, uint64_t *bsum,
                          const DevTables *tabs, uint32_t *crc_out, unsigned ncu, hipStream_t st,
                          hipEvent_t ev0, hipEvent_t ev1);
// chain_cap > 0 (batches with big files offloaded): when big_plan_kernel's
// *nbig is at most chain_cap / 4 (one per CU), each big file's MD5 runs on a
// workgroup of its own (md5_chain_wg, fdfs_md5.hip), up to chain_cap (one
// per SIMD) on a wave of its own (md5_chain_wave).  launch_sig_hash: up to
// chain_cap (one per CU) ELF chains on workgroups of their own.
hipError_t launch_md5_stage(bool sar, const uint8_t *base, const uint64_t *offs,
                            const uint64_t *sizes, uint32_t n, const uint32_t *order,
                            const DevTables *tabs, const uint64_t *big_min, uint32_t *queue, uint32_t *crc_out,
                            uint8_t *sig_out, int32_t *codes_out, fdfs_gpu_file_state *states,
                            const uint32_t *sidx, unsigned ncu, hipStream_t st,
                            const uint32_t *nbig = nullptr, uint32_t chain_cap = 0);
// CRC32 only, one lane per file of a size-binned order (large batches of
// files below *big_min; fdfs_hash.hip crc_lane_kernel).
hipError_t launch_crc_lane(bool sar, const uint8_t *base, const uint64_t *offs, const uint64_t *sizes, uint32_t n,
                           const uint32_t *order, const DevTables *tabs, const uint64_t *big_min, uint32_t *crc_out,
                           hipStream_t st);
hipError_t launch_sig_hash(bool sar, const uint8_t *base, const uint64_t *offs,
                           const uint64_t *sizes, uint32_t n, const uint32_t *order,
                           const DevTables *tabs, const uint64_t *big_min, uint32_t *crc_out, uint8_t *sig_out,
                           int32_t *codes_out, fdfs_gpu_file_state *states, const uint32_t *sidx,
                           hipStream_t st, const uint32_t *nbig = nullptr, uint32_t chain_cap = 0);

// chunked-update helpers (fdfs_stream.hip)
hipError_t launch_state_init(fdfs_gpu_file_state *states, uint32_t n, hipStream_t st);
// CRC_ONLY update: crc[f] = CRC32_FINAL(CRC32_ex(chunk f, XINIT)) from
// crc_seg_kernel, carried onto the chunk's state (and its count advanced).
hipError_t launch_crc_carry(const uint32_t *crc, const uint64_t *sizes, uint32_t n,
                            const uint32_t *sidx, fdfs_gpu_file_state *states, const DevTables *tabs,
                            hipStream_t st);
hipError_t launch_final(int method, const fdfs_gpu_file_state *states, const uint32_t *sidx,
                        uint32_t n, uint32_t *crc_out, uint8_t *sig_out, int32_t *codes_out,
                        hipStream_t st);
hipError_t launch_crc_combine(const uint32_t *a, const uint32_t *b, const uint64_t *len_b, uint32_t n,
                              uint32_t *out, const DevTables *tabs, hipStream_t st);
// Split-file CRC: one rank's block of per-file words is {CRC term u32 x
// nfiles, error word, length sum u64 x nfiles, boundary sum u64 x nfiles};
// `base` is rank 0's block and rank r's starts `stride` bytes further per
// rank (the all-gather's layout).
struct CrcParts {
    char *base;
    uint64_t nfiles, stride;
    static uint64_t err_off(uint64_t nfiles) { return (4 * nfiles + 7) & ~7ull; }
    static uint64_t block_bytes(uint64_t nfiles) { return err_off(nfiles) + 8 + 16 * nfiles; }
    __host__ __device__ uint32_t *word(uint32_t r, uint64_t f) const
    {
        return reinterpret_cast<uint32_t *>(base + r * stride) + f;
    }
    __host__ __device__ uint32_t *err(uint32_t r) const
    {
        return reinterpret_cast<uint32_t *>(base + r * stride + ((4 * nfiles + 7) & ~7ull));
    }
    __host__ __device__ uint64_t *len(uint32_t r, uint64_t f) const
    {
        return reinterpret_cast<uint64_t *>(base + r * stride + ((4 * nfiles + 7) & ~7ull) + 8) + f;
    }
    // sum over the file's pieces of H(end) - H(start) (mod 2^64): equals
    // H(size) - H(0) exactly when the pieces tile the file (see crc_piece_kernel)
    __host__ __device__ uint64_t *bnd(uint32_t r, uint64_t f) const
    {
        return reinterpret_cast<uint64_t *>(base + r * stride + ((4 * nfiles + 7) & ~7ull) + 8) + nfiles + f;
    }
};
// Each piece's term XORed into its rank's block (launch_crc_pieces), then
// the fold of nranks blocks into the files' CRCs, the mask of ranks that
// reported an error (err_out[0]) and the count of files whose pieces do not
// tile them exactly (err_out[1], zeroed by the caller).
hipError_t launch_crc_pieces(const uint32_t *crc, const uint64_t *pfile, const uint64_t *pstart, const uint64_t *plen,
                             uint32_t np, const uint64_t *fsize, uint64_t nfiles, const CrcParts &blk,
                             const DevTables *tabs, hipStream_t st);
hipError_t launch_crc_fold(const CrcParts &blk, uint32_t nranks, const uint64_t *fsize, uint64_t nfiles,
                           uint32_t *crc_out, uint64_t *err_out, const DevTables *tabs, hipStream_t st);
// Duplicate state indices of an update batch: *flag = 1 duplicate, 2 the
// reserved value ~0 (table: sidx_table_size(n) u32 of scratch).
uint32_t sidx_table_size(uint32_t n);
hipError_t launch_sidx_check(const uint32_t *sidx, uint32_t n, uint32_t *table, uint32_t *flag, hipStream_t st);
int crc_seg_blocks_per_cu();  // the fold kernel (crc_seg_kernel)
int crc_tab_blocks_per_cu();  // the table kernel (crc_tab_kernel)

// formats, FastDHT routing, scrub (fdfs_format.hip)
hipError_t launch_file_ids(bool sar, uint32_t server_id, const uint32_t *crc32, const int64_t *size,
                           const int32_t *ts, const uint32_t *rnd, uint32_t n, uint32_t subdirs,
                           char *name_out, uint8_t *sub_out, hipStream_t st);
hipError_t launch_parse_file_ids(const uint8_t *names, uint32_t n, uint32_t *sid, int32_t *ts,
                                 int64_t *size, uint32_t *crc, hipStream_t st);
hipError_t launch_trunk_pack(const uint8_t *type, const int32_t *alloc, const int32_t *size,
                             const uint32_t *crc, const int32_t *mtime, const uint8_t *ext,
                             uint32_t n, uint8_t *hdr, hipStream_t st);
hipError_t launch_trunk_unpack(const uint8_t *hdr, uint32_t n, uint8_t *type, int32_t *alloc,
                               int32_t *size, uint32_t *crc, int32_t *mtime, uint8_t *ext,
                               hipStream_t st);
uint32_t pjw_prefix(bool sar, const char *ns, int len);
hipError_t launch_fdht_route(bool sar, const uint8_t *keys, uint32_t stride, const uint32_t *lens,
                             uint64_t n, const uint64_t *dcount, uint32_t h0, uint32_t group_count,
                             const uint32_t *servers, int32_t *hash_out, uint32_t *group_out,
                             uint32_t *server_out, uint32_t *gcount, uint64_t *start,
                             uint64_t *cursor, uint64_t *order, hipStream_t st);
hipError_t launch_sources(const uint64_t *rep, uint64_t n, const uint8_t *sig, const uint8_t *ids,
                          uint32_t stride, const uint32_t *lens, uint64_t *flag, uint64_t *pos,
                          uint64_t *bsum, uint64_t *iota, uint64_t *index, uint8_t *csig,
                          uint8_t *cids, uint32_t *clens, uint64_t *nsrc, hipStream_t st);
hipError_t launch_scrub(const uint32_t *crc, const uint32_t *expect, uint32_t n, uint8_t *bad,
                        uint32_t *nbad, hipStream_t st);

// dedup path (fdfs_dedup.hip)
uint64_t dedup_ws_bytes(uint64_t n);

// fdfs_gpu_dedup_global's owner side: only the records of multi-member
// classes are answered, as 16-byte records {sender row, ref, rep lo, rep hi}
// appended per segment of the owner's received rows (fdfs_dedup.hip DpSink).
// seg: seg_start[0 .. nseg] (rows), then at seg + kSinkSoff the segments'
// first rows in their senders' send order; written by launch_sink_plan.
constexpr int kSinkSoff = 65;
constexpr int kSinkSegWords = 2 * 65;
struct DedupSink {
    void *ans;            // uint4[rows]: segment k's records from ans + seg_start[k]
    uint32_t *cntr;       // [64] records per segment
    const uint64_t *seg;  // [kSinkSegWords]
    uint32_t nseg;
};
// The source rank of segment k of owner q's received rows: its own rows
// first (the bucket pass writes them in place), then the others in rank order.
__host__ __device__ inline uint32_t dg_seg_src(uint32_t q, uint32_t k) { return k == 0 ? q : (k <= q ? k - 1 : k); }
// launch_dedup_bucket's extras for fdfs_gpu_dedup_global (all optional):
// rows of owner `me` straight into self_rows (the owner-side buffer), the
// record of each send position, every record's singleton answer pre-filled.
struct BucketExtra {
    uint32_t me;
    uint8_t *self_rows;
    uint32_t *rec_of;
    uint64_t *rep_out;
    uint32_t *ref_out;
};

// packed: rep_out is an array of 16-byte {rep, ref, 0} records (ref_out unused);
// xs: answers as sink records instead (rep_out / ref_out unused)
hipError_t launch_dedup_group(const uint8_t *sig, uint32_t sig_stride, const uint64_t *gidx,
                              uint32_t gidx_stride, uint64_t n, void *ws, uint64_t *rep_out,
                              uint32_t *ref_out, bool packed, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1,
                              const DedupSink *xs = nullptr);
hipError_t launch_dedup_bucket(const uint8_t *sig, const uint64_t *gidx, uint64_t n,
                               uint32_t nranks, uint8_t *records_out, uint64_t *counts_out,
                               uint64_t *ws, uint64_t *row_of_out, hipStream_t st,
                               hipEvent_t ev0, hipEvent_t ev1, const BucketExtra *extra = nullptr);
// fdfs_gpu_dedup_global's one-pass bucket: owner q's rows at [q cap, q cap +
// counts[q]) of the send order (rows past cap not written: counts[q] > cap
// tells the plan to bucket again with launch_dedup_bucket); x.rec_of,
// x.rep_out and x.ref_out required.
uint64_t bucket_cap(uint64_t n, uint32_t nranks);
hipError_t launch_bucket_place(const uint8_t *sig, const uint64_t *gidx, uint64_t n, uint32_t nranks,
                               uint64_t cap, uint8_t *rows, uint64_t *counts, const BucketExtra &x, hipStream_t st,
                               hipEvent_t ev0, hipEvent_t ev1);
// exact: every sender used the exact prefix layout (a rebucket after an
// over-capacity owner), not its announced cap
hipError_t launch_sink_plan(const uint64_t *ann, uint32_t w, uint32_t nranks, uint32_t q, bool exact, uint64_t *seg,
                            uint32_t *cntr, hipStream_t st);
// na: device count of list a (<= na_max records); nb: host count of list b
hipError_t launch_answer_apply(const void *a, const uint32_t *na, uint64_t na_max, const void *b, uint64_t nb,
                               const uint32_t *rec_of, uint64_t *rep_out, uint32_t *ref_out, hipStream_t st);
// u64 words of launch_dedup_bucket's workspace for n records
size_t bucket_ws_elems(uint64_t n);

// incremental dedup index (fdfs_index.hip)
struct IndexTable {
    uint64_t slots;       // power of two
    uint8_t *keys;        // [slots][24] signatures
    uint64_t *rep;        // [slots] class source (ingest index)
    uint32_t *ref;        // [slots] class size so far
    uint32_t *state;      // [slots] empty / busy / full
    uint64_t *counters;   // [4]: classes, -, unplaced classes (table full), -
};
hipError_t launch_index_clear(uint32_t *state, uint64_t slots, hipStream_t st);
hipError_t launch_index_rehash(const IndexTable &from, const IndexTable &to, hipStream_t st);
hipError_t launch_index_ingest(const uint8_t *sig, const uint64_t *gidx, uint64_t gbase, uint64_t n,
                               const uint64_t *rep_pos, const uint32_t *ref_b, const IndexTable &t,
                               uint64_t *res_rep, uint32_t *res_ref, uint64_t *rep_out, uint32_t *ref_out,
                               hipStream_t st);

hipError_t launch_answer_gather(const uint64_t *back, const uint64_t *row_of, uint64_t n, uint64_t *rep_out,
                                uint32_t *ref_out, hipStream_t st);

}  // namespace fdfs
