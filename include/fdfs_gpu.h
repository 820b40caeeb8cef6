/*
 * fdfs_gpu.h -- C ABI of libfdfs_gpu: MI355X (gfx950) batch implementation of
 * FastDFS's upload-path CRC32 + duplicate-check signature, and of the bulk
 * duplicate grouping that replaces per-file FastDHT lookups.
 *
 * Plain C types only: device pointers are `const void *` / `void *`, streams
 * are hipStream_t passed as `void *` (NULL = the null stream).
 *
 * Threading: a context serialises its calls (a mutex; any host thread may
 * call), and the device workspace it owns is ordered across streams: a call
 * on stream B starts after the previous call of the context, on stream A,
 * has finished with it.  Calls stay asynchronous on their stream.  Inside a
 * hipStream capture this cross-stream ordering is not recorded, so a
 * captured sequence must use one stream, after fdfs_gpu_reserve.  For
 * concurrency across dio threads, open one context per thread.  Every call
 * returns 0 or a positive errno value (EINVAL bad arguments, ENOMEM
 * allocation failure, EIO a HIP error), the convention of the reference's
 * storage daemon (e.g. storage/storage_dio.c:443).  Inputs are caller owned
 * and never modified; outputs are preallocated by the caller.
 *
 * Interfaces replaced (reference file:line -> entry point):
 *   CRC32_XINIT / CRC32_ex / CRC32_FINAL
 *       storage/storage_service.c:7149, storage/storage_dio.c:467,500,
 *       client/fdfs_crc32.c:67,91,99           -> fdfs_gpu_sig_batch(.., FDFS_SIG_CRC_ONLY, ..)
 *   INIT/CALC/FINISH_HASH_CODES4 + STORAGE_GEN_FILE_SIGNATURE
 *       storage/storage_service.c:7156, storage/storage_dio.c:475,508,
 *       storage/storage_service.c:106-120,2635 -> fdfs_gpu_sig_batch(.., FDFS_SIG_HASH, ..)
 *   my_md5_init/update/final + STORAGE_GEN_FILE_SIGNATURE
 *       storage/storage_service.c:7160, storage/storage_dio.c:480,512  -> fdfs_gpu_sig_batch(.., FDFS_SIG_MD5, ..)
 *   fdht_get_ex1 "fid" / fdht_set_ex / fdht_inc_ex "ref" dedup decision
 *       storage/storage_service.c:2652,2714,2734,2984 -> fdfs_gpu_dedup (1 GPU),
 *       fdfs_gpu_dedup_global (N GPUs over RCCL), or fdfs_gpu_dedup_bucket +
 *       the caller's exchange + fdfs_gpu_dedup_group
 *   the per-chunk loop itself (StorageFileContext state across chunks)
 *       storage/storage_service.c:7147-7161, storage/storage_dio.c:465-515,
 *       client/fdfs_crc32.c:67-99 -> fdfs_gpu_state_init / fdfs_gpu_update_batch /
 *       fdfs_gpu_final_batch (+ fdfs_gpu_crc_combine for pieces hashed apart)
 *   storage_gen_filename + storage_get_store_path (random mode)
 *       storage/storage_service.c:2080-2202      -> fdfs_gpu_file_ids
 *   fdfs_get_file_info_ex's name decode
 *       client/storage_client.c:2133-2214        -> fdfs_gpu_parse_file_ids
 *   trunk_pack_header / trunk_unpack_header
 *       storage/trunk_mgr/trunk_shared.c:340-370 -> fdfs_gpu_trunk_pack / _unpack
 *   CALC_KEY_HASH_CODE + group / server pick of the dedup keys
 *       storage/fdht_client/fdht_client.c:207-212,256-305,375-376 -> fdfs_gpu_fdht_route,
 *       fdfs_gpu_fdht_route_keys
 *   (new) CRC scrub of stored files against their file-id CRCs -> fdfs_gpu_scrub
 *   recovery / sync-receiver batch mode (storage/storage_disk_recovery.c:512-761,
 *       storage/storage_service.c:5468-5779)  -> fdfs_gpu_recovery_batch
 */
#ifndef FDFS_GPU_H
#define FDFS_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FDFS_GPU_ABI_VERSION 1

/* Signature methods: values of STORAGE_FILE_SIGNATURE_METHOD_*
 * (storage/storage_global.h:41-42); 0 = CRC32 only (check_file_duplicate=0,
 * conf/storage.conf:195). */
#define FDFS_SIG_CRC_ONLY 0
#define FDFS_SIG_HASH     1
#define FDFS_SIG_MD5      2

#define FDFS_FILE_SIGNATURE_SIZE 24   /* storage/storage_service.c:106 */

/* Context flags. */
/* CRC32_ex / ELFHash_ex with an unsigned state (logical >>).  The default
 * (flag clear) is the signed-int state libfastcommon declares (arithmetic >>),
 * see DESIGN.md "Oracle" for why both exist. */
#define FDFS_GPU_FLAG_UNSIGNED_HASH 0x1u

typedef struct fdfs_gpu_ctx fdfs_gpu_ctx;

/* A batch of files in device memory: file i is bytes
 * [base + offset[i], base + offset[i] + size[i]).  offset/size are device
 * arrays of n entries.  Files may start at any byte (measured: byte-packed
 * batches hash at the rate of 16-byte aligned ones). */
typedef struct {
    const void     *base;
    const uint64_t *offset;
    const uint64_t *size;
    uint32_t        n;
} fdfs_gpu_batch;

/* Version / capability probe; returns FDFS_GPU_ABI_VERSION. */
int fdfs_gpu_abi_version(void);

/* Open a context on HIP device `device`: builds and uploads the CRC tables
 * for the selected hash semantics.  *out receives the handle. */
int fdfs_gpu_open(int device, unsigned flags, fdfs_gpu_ctx **out);
int fdfs_gpu_close(fdfs_gpu_ctx *ctx);

/* Reserve device workspace for batches of up to max_files files and
 * dedup of up to max_records records, so later calls do no allocation
 * and issue no host synchronisation: a fixed-shape sequence of calls on one
 * stream can then be captured in a hipGraph and replayed
 * (tests/test_gpu_graph.py: sig_batch of every method + dedup, replayed
 * over changing bytes).  Optional: calls grow it on demand. */
int fdfs_gpu_reserve(fdfs_gpu_ctx *ctx, uint64_t max_files, uint64_t max_records);

/* Per-file CRC32 (always, as uploads do: storage/storage_service.c:4533) and,
 * for FDFS_SIG_HASH / FDFS_SIG_MD5, the 24-byte duplicate-check signature.
 *   crc_out:   device uint32_t[n], the %u value fdfs_crc32 prints.
 *   sig_out:   device uint8_t[n*24] or NULL (ignored for CRC_ONLY).
 *   codes_out: device int32_t[n*4] or NULL: file_hash_codes after FINISH
 *              (HASH) or the raw MD5 digest (MD5), as StorageFileContext holds
 *              them (storage/storage_nio.h:94).
 * Asynchronous on `stream`. */
int fdfs_gpu_sig_batch(fdfs_gpu_ctx *ctx, const fdfs_gpu_batch *batch, int method,
                       uint32_t *crc_out, uint8_t *sig_out, int32_t *codes_out,
                       void *stream);

/* The same for a batch in HOST memory (the daemon's receive buffers, the
 * CLI's files): base/offset/size are host pointers, crc_out / sig_out /
 * codes_out host arrays.  Files are streamed to the device in windows of at
 * most chunk_bytes (0 = 256 MiB), double-buffered on two internal streams
 * (window k+1 crosses PCIe while window k is hashed); a file larger than the
 * space left in a window continues in the next one, its state carried on the
 * device (the chunked path below), so device memory is two windows plus
 * 172 bytes per file whatever the file sizes.  Synchronous: returns when
 * every result is in host memory.  A pinned base (hipHostMalloc /
 * hipHostRegister) copies at the full PCIe rate; batches with increasing
 * offsets copy each byte once. */
int fdfs_gpu_sig_batch_host(fdfs_gpu_ctx *ctx, const fdfs_gpu_batch *host_batch, int method,
                            uint32_t *crc_out, uint8_t *sig_out, int32_t *codes_out,
                            uint64_t chunk_bytes);

/* ---- Chunked (state-carrying) form of the same path ---------------------
 * The storage daemon hashes an upload one received chunk at a time
 * (<= buff_size, conf/storage.conf:52) and keeps the running values in the
 * file's StorageFileContext (storage/storage_nio.h:94-96):
 *     storage_write_to_file   init   (storage/storage_service.c:7147-7161)
 *     dio_write_file          update (storage/storage_dio.c:465-483)
 *                             final  (storage/storage_dio.c:498-515)
 * These three calls are that loop for a batch of uploads at once: each call
 * advances many files by one chunk each, on the GPU.  The state is a device
 * array of fdfs_gpu_file_state laid out as StorageFileContext holds it
 * (int crc32; int file_hash_codes[4]; MD5_CTX {state[4], count[2],
 * buffer[64]}); it can be saved, moved between calls and streams, and
 * resumed.  Results equal the one-shot fdfs_gpu_sig_batch over the
 * concatenated chunks for every chunking. */
typedef struct {
    int32_t  crc32;          /* CRC32_ex running value (CRC32_XINIT at init) */
    int32_t  hash_codes[4];  /* CALC_HASH_CODES4 running values (FDFS_SIG_HASH) */
    uint32_t md5_state[4];   /* MD5_CTX.state (FDFS_SIG_MD5) */
    uint32_t md5_count[2];   /* bits hashed so far, low word first (MD5_CTX.count);
                                kept for every method: the signature's file size */
    uint8_t  md5_buffer[64]; /* MD5_CTX.buffer: the (count / 8) % 64 pending bytes */
    uint8_t  reserved[20];
} fdfs_gpu_file_state;       /* 128 bytes */

/* storage_write_to_file's initialisation of n states (device array):
 * crc32 = CRC32_XINIT, INIT_HASH_CODES4, my_md5_init, count 0. */
int fdfs_gpu_state_init(fdfs_gpu_ctx *ctx, fdfs_gpu_file_state *states, uint32_t n, void *stream);

/* dio_write_file's per-chunk update for a batch of chunks (device memory):
 * chunk i = bytes [base + offset[i], + size[i]) is hashed onto
 * states[state_idx ? state_idx[i] : i]: CRC32_ex always (as uploads do,
 * storage/storage_service.c:4533), CALC_HASH_CODES4 for FDFS_SIG_HASH,
 * my_md5_update for FDFS_SIG_MD5.  A state may appear at most once per call
 * (the daemon has one chunk of an upload in flight at a time): with
 * state_idx given, the call checks this first (one small kernel and a host
 * synchronisation) and returns EINVAL without touching any state on a
 * repeated index or the reserved index 0xFFFFFFFF (inside a stream capture
 * the check is skipped and the contract is the caller's; with state_idx the
 * checked call takes at most 2^30 chunks, EINVAL above).  Chunks may start
 * at any byte and have any length, including 0. */
int fdfs_gpu_update_batch(fdfs_gpu_ctx *ctx, const fdfs_gpu_batch *chunks, const uint32_t *state_idx,
                          int method, fdfs_gpu_file_state *states, void *stream);

/* dio_write_file's finalisation for n files: CRC32_FINAL (crc_out[i], the
 * %u value), FINISH_HASH_CODES4 or my_md5_final, and
 * STORAGE_GEN_FILE_SIGNATURE with file size = bytes hashed (sig_out[i],
 * codes_out[i]; either may be NULL) of states[state_idx ? state_idx[i] : i].
 * The states are not modified. */
int fdfs_gpu_final_batch(fdfs_gpu_ctx *ctx, const fdfs_gpu_file_state *states,
                         const uint32_t *state_idx, uint32_t n, int method, uint32_t *crc_out,
                         uint8_t *sig_out, int32_t *codes_out, void *stream);

/* crc32_combine: out[i] = the CRC32_ex running value of A || B given
 * crc_a[i] = CRC32_ex(A, init) and crc_b[i] = CRC32_ex(B, 0), with len_b[i] =
 * |B| (device arrays): M^(8 |B|) crc_a XOR crc_b over GF(2).  Joins the
 * partial states of one file hashed in pieces on several GPUs. */
int fdfs_gpu_crc_combine(fdfs_gpu_ctx *ctx, const uint32_t *crc_a, const uint32_t *crc_b,
                         const uint64_t *len_b, uint32_t n, uint32_t *out, void *stream);

/* Single-GPU duplicate grouping over n records in ingest order.
 *   sig:  device uint8_t[n*24]; gidx: device uint64_t[n] global ingest index
 *         of each record, or NULL for 0..n-1.
 *   rep_out: device uint64_t[n], ingest index of the class's first file
 *            (the FastDHT "fid" source, storage/storage_service.c:2714).
 *   ref_out: device uint32_t[n], class size (the "ref" count after all
 *            links, storage/storage_service.c:2734,2984). */
int fdfs_gpu_dedup(fdfs_gpu_ctx *ctx, const uint8_t *sig, const uint64_t *gidx,
                   uint64_t n, uint64_t *rep_out, uint32_t *ref_out, void *stream);

/* The same answers packed, one 16-byte record per input record: rep and ref
 * of a record share a cache line, so the group's random answer stores
 * dirty one line per record instead of two (and the singleton answers are
 * one 16-byte store).  out: device fdfs_gpu_dedup_answer[n], 16-byte aligned
 * (EINVAL otherwise). */
typedef struct {
    uint64_t rep;       /* as rep_out of fdfs_gpu_dedup */
    uint32_t ref;       /* as ref_out */
    uint32_t reserved;  /* written 0 */
} fdfs_gpu_dedup_answer;
int fdfs_gpu_dedup_packed(fdfs_gpu_ctx *ctx, const uint8_t *sig, const uint64_t *gidx, uint64_t n,
                          fdfs_gpu_dedup_answer *out, void *stream);

/* Multi-GPU dedup building blocks (one process per GPU; the exchange between
 * the two calls is the caller's all-to-all over RCCL/xGMI).
 * Bucket: packs records {sig[24], gidx (uint64 LE)} into 32-byte rows grouped
 * by owner rank (owner = hash(sig) mod nranks, nranks <= 64):
 *   records_out: device uint8_t[n*32], rows of owner 0 first, then owner 1 ..
 *   counts_out:  device uint64_t[nranks], rows per owner;
 *   row_of_out:  device uint64_t[n] or NULL, row index of record i (to route
 *                the owner's answers back). */
int fdfs_gpu_dedup_bucket(fdfs_gpu_ctx *ctx, const uint8_t *sig, const uint64_t *gidx,
                          uint64_t n, uint32_t nranks, uint8_t *records_out,
                          uint64_t *counts_out, uint64_t *row_of_out, void *stream);
/* Group: the owner's records (n rows of 32 B, device) -> per-row rep (min gidx
 * of its class) and ref (class size), in row order. */
int fdfs_gpu_dedup_group(fdfs_gpu_ctx *ctx, const uint8_t *records, uint64_t n,
                         uint64_t *rep_out, uint32_t *ref_out, void *stream);

/* Incremental dedup across ingest batches: a device-resident signature ->
 * {source, ref} table that persists between calls, i.e. the FastDHT state
 * the upload path builds one RPC at a time (storage/storage_service.c:2652
 * "fid" get, :2714 set on a miss, :2734 / :2984 "ref"), kept in HBM.
 * fdfs_gpu_index_ingest takes the next batch of an ingest stream (records in
 * ingest order; gidx: their global ingest indices, increasing across
 * batches, or NULL for the index's own running count) and returns for each
 * record rep_out = the ingest index of the first file EVER ingested with its
 * signature (an earlier batch's source stays the source) and ref_out = the
 * class size once this batch is in.  After k batches the answers equal
 * fdfs_gpu_dedup over the concatenation of all k.  max_classes sizes the
 * table (load <= 3/4, 40 bytes per slot); it is not a limit: when a batch
 * might not fit (a host-side bound of the classes so far plus the batch's
 * records, refined by reading back the exact count, one synchronisation),
 * the table grows to twice its slots until it fits and every class is
 * rehashed into it, before the batch is grouped.  So every class of every
 * batch is placed: no answer is ever given "within its batch only".  If the
 * growth cannot be allocated, ingest returns ENOMEM and the index is
 * unchanged (the batch was not ingested; ENOSPC if growth is needed inside a
 * stream capture).  fdfs_gpu_index_stats is synchronous (waits for the last
 * ingest); unplaced stays 0.  Ingests into one index are ordered whatever
 * their streams; ingest, stats, slots and destroy of one index may be called
 * from any thread (the index has its own lock). */
typedef struct fdfs_gpu_index fdfs_gpu_index;
int fdfs_gpu_index_create(fdfs_gpu_ctx *ctx, uint64_t max_classes, fdfs_gpu_index **out);
int fdfs_gpu_index_destroy(fdfs_gpu_index *index);
int fdfs_gpu_index_ingest(fdfs_gpu_ctx *ctx, fdfs_gpu_index *index, const uint8_t *sig,
                          const uint64_t *gidx, uint64_t n, uint64_t *rep_out, uint32_t *ref_out,
                          void *stream);
int fdfs_gpu_index_stats(fdfs_gpu_index *index, uint64_t *classes, uint64_t *records,
                         uint64_t *unplaced);
/* The table's current slot count (grows as above). */
int fdfs_gpu_index_slots(fdfs_gpu_index *index, uint64_t *slots);

/* Multi-GPU dedup in one call, over RCCL (xGMI between the GPUs of a node):
 * one process per GPU, each holding its share of the ingest (sig, gidx: the
 * files' global ingest indices, required when the communicator has more
 * than one rank); every rank calls it with its share and gets rep_out /
 * ref_out for its own records, identical to fdfs_gpu_dedup over the
 * concatenated ingest.  Inside: bucket by owner rank (the FastDHT key
 * partition, storage/fdht_client/fdht_client.c:301-305, as a GPU bucket),
 * which also writes every record's singleton answer (rep = its gidx, ref =
 * 1) and puts the rank's own rows straight into its owner-side buffer; one
 * ncclAllGather of every rank's announcement (rows per owner, the room of
 * its owner-side buffers, any local error), from which every rank derives
 * the same exchange plan; grouped ncclSend/ncclRecv of the 32-byte rows to
 * the other owners; the owner's group, which answers only the rows of
 * multi-member classes (16-byte records {sender row, ref, rep}); one small
 * ncclAllGather of those records' counts; the records sent back the same
 * way and applied over the singleton answers.  Host synchronisations: the
 * announcement (the row exchange is sized by it) and, with more than one
 * rank, the record counts (the way back is sized by them), plus one small
 * all-reduce when some owner's buffers must grow.
 * Errors: an argument error or allocation failure on ANY rank is returned by
 * EVERY rank (EINVAL / ENOMEM; fdfs_gpu_last_error names the rank) before
 * any row moves, so no rank is left waiting.  EIO after that point (a failed
 * launch or RCCL call) leaves the communicator unusable: abort it.  Not
 * capturable (it synchronises on the announcements): inside a stream capture
 * it returns EINVAL before any collective is enqueued; every rank must call
 * it outside a capture.
 * comm: an ncclComm_t (RCCL) of the ranks taking part, each rank's
 * communicator on this context's device.  Replaces the per-file
 * fdht_get_ex1 / fdht_set_ex / fdht_inc_ex round trips
 * (storage/storage_service.c:2652,2714,2734,2984) for bulk ingest. */
int fdfs_gpu_dedup_global(fdfs_gpu_ctx *ctx, void *comm, const uint8_t *sig, const uint64_t *gidx,
                          uint64_t n, uint64_t *rep_out, uint32_t *ref_out, void *stream);

/* fdfs_gpu_dedup_global for `nranks` VIRTUAL ranks in this process, all on
 * this context's device: rank p's share is sig[p], gidx[p], n[p] -> rep_out[p],
 * ref_out[p] (host arrays of nranks device pointers / counts).  It runs the
 * same bucket, exchange plan, group, sink and apply code as the RCCL form;
 * every (src, dst) segment moves by hipMemcpyAsync where RCCL would send it.
 * This is how the multi-rank offsets and answer routing are checked on one
 * GPU (tests/test_gpu_dedup.py), and a one-process fallback for a caller
 * that holds every share.  Synchronous; allocates its exchange buffers. */
int fdfs_gpu_dedup_global_local(fdfs_gpu_ctx *ctx, int nranks, const uint8_t *const *sig,
                                const uint64_t *const *gidx, const uint64_t *n, uint64_t *const *rep_out,
                                uint32_t *const *ref_out, void *stream);

/* Bytes the context's last fdfs_gpu_dedup_global(_local) call moved between
 * ranks (sent by this rank; all virtual ranks for _local): the 32-byte rows
 * to the other owners, and the 16-byte answer records back to the other
 * ranks.  Measurement only (bench.py's xGMI bytes per step). */
int fdfs_gpu_dedup_global_stats(fdfs_gpu_ctx *ctx, uint64_t *row_bytes, uint64_t *answer_bytes);

/* Split-file CRC32 over N GPUs: the bytes of `nfiles` files
 * are spread over the ranks in pieces, cut anywhere (e.g. the files'
 * concatenated byte stream in equal shares, fastdfs_amd/dist.py
 * plan_crc_pieces: a recovery or scrub pass over a few huge files keeps
 * every GPU busy).  Each rank passes the pieces it holds as a batch (piece
 * i = bytes [base + offset[i], + size[i]) on this rank's device) with
 * piece_file[i] (the file it belongs to) and piece_start[i] (its first
 * byte's position in that file), device uint64 arrays of pieces->n entries;
 * file_size: device uint64[nfiles], the same on every rank.  Every rank gets
 * crc_out (device uint32[nfiles]) = the CRC32 (%u value) of every file.
 * Inside: CRC32_ex of every piece from CRC32_XINIT (the segmented kernel),
 * each piece's CRC32_ex(piece, 0) advanced to the end of its file by a
 * GF(2) power of the zero-byte step and XORed into a per-file word, one
 * ncclAllGather of those words (20 bytes per file per rank), and the fold
 * M^size CRC32_XINIT ^ (the ranks' words), then CRC32_FINAL -- CRC32_ex is
 * linear over GF(2), so pieces may come in any order from any rank (the
 * reference's CRC32_ex(.., init) chaining, storage/storage_dio.c:467,
 * client/fdfs_crc32.c:67-99, computed for the pieces apart).  The pieces of
 * all ranks must tile each file exactly: a piece outside its file, or a file
 * whose pieces do not tile it (lengths that do not add up to its size, or
 * overlaps and gaps: checked by a sum of H(end) - H(start) over its pieces,
 * H a 64-bit position hash, against H(size) - H(0)), makes every rank return
 * EINVAL (crc_out invalid).  An argument error or allocation failure on ANY
 * rank is returned by every rank (first, an all-gather of {nfiles, errno},
 * one host synchronisation).  Synchronous: returns after crc_out is written
 * (a second synchronisation reads the ranks' error words).  Not capturable:
 * called inside a stream capture it returns EINVAL before any collective is
 * enqueued (a captured collective would not run, so no rank could be told);
 * every rank must call it outside a capture.  EIO (a failed launch or RCCL
 * call) leaves the communicator unusable. */
int fdfs_gpu_crc_batch_global(fdfs_gpu_ctx *ctx, void *comm, const fdfs_gpu_batch *pieces,
                              const uint64_t *piece_file, const uint64_t *piece_start,
                              const uint64_t *file_size, uint64_t nfiles, uint32_t *crc_out, void *stream);

/* fdfs_gpu_crc_batch_global for `nranks` VIRTUAL ranks in this process, all
 * on this context's device: pieces[p], piece_file[p], piece_start[p] are
 * virtual rank p's (host arrays of nranks entries, device data), crc_out the
 * one result.  The same per-rank blocks and fold as the RCCL form, each
 * block written where the all-gather would put it. */
int fdfs_gpu_crc_batch_global_local(fdfs_gpu_ctx *ctx, int nranks, const fdfs_gpu_batch *pieces,
                                    const uint64_t *const *piece_file, const uint64_t *const *piece_start,
                                    const uint64_t *file_size, uint64_t nfiles, uint32_t *crc_out, void *stream);

/* Convenience RCCL communicator setup for callers without one: rank 0 gets
 * a 128-byte id (ncclGetUniqueId) and sends it to the others by any means;
 * every rank then calls fdfs_gpu_comm_init (ncclCommInitRank on ctx's
 * device; collective: all ranks at once). */
#define FDFS_GPU_COMM_ID_BYTES 128
int fdfs_gpu_comm_unique_id(uint8_t *id_out);
int fdfs_gpu_comm_init(fdfs_gpu_ctx *ctx, const uint8_t *id, int nranks, int rank, void **comm_out);
int fdfs_gpu_comm_destroy(void *comm);

/* Kernel timing (for benchmarks and profiling).  When enabled, every call
 * records a HIP event pair on its stream around its main kernel:
 *   FDFS_KERNEL_SIG_LANE  sig_hash_kernel / md5_pair_kernel (md5_stage_kernel for
 *                         update_batch) (FDFS_SIG_HASH / FDFS_SIG_MD5)
 *   FDFS_KERNEL_CRC_SEG   the CRC-only kernels (FDFS_SIG_CRC_ONLY): crc_tab_kernel +
 *                         crc_seg_kernel, or for batches of more than three
 *                         waves per SIMD of files crc_seg_kernel (files >= 96 KiB)
 *                         + crc_lane_kernel (the rest)
 *   FDFS_KERNEL_DEDUP     dp_tile .. dp_group_slow, the whole grouping chain (fdfs_gpu_dedup / _group)
 *   FDFS_KERNEL_BUCKET    count + scatter   (fdfs_gpu_dedup_bucket)
 * fdfs_gpu_read_timing waits for the recorded events, returns the summed
 * milliseconds and launch count for `kernel` since the last read, and resets
 * them. */
#define FDFS_KERNEL_SIG_LANE 0
#define FDFS_KERNEL_CRC_SEG  1
#define FDFS_KERNEL_DEDUP    2
#define FDFS_KERNEL_BUCKET   3
int fdfs_gpu_set_timing(fdfs_gpu_ctx *ctx, int enable);
int fdfs_gpu_read_timing(fdfs_gpu_ctx *ctx, int kernel, double *ms_out, uint64_t *launches_out);

/* The CRC-only batch size above which fdfs_gpu_sig_batch hashes the files
 * below 96 KiB one lane per file (crc_lane_kernel) instead of a wave per
 * file: more than min_files files (three waves per SIMD of this device,
 * kCrcLaneMinFill x CUs x 256).  Measurement only: bench.py names the kernel
 * its CRC-only line times from it. */
int fdfs_gpu_crc_lane_min_files(fdfs_gpu_ctx *ctx, uint64_t *min_files);

/* ---- Formats that consume the file CRC, FastDHT routing, scrub ---------- */

#define FDFS_FILENAME_BASE64_LENGTH 27  /* tracker/tracker_types.h:35 */
#define FDFS_TRUNK_HEADER_SIZE      24  /* storage/trunk_mgr/trunk_shared.h:40 */
#define FDFS_EXT_NAME_FIELD         7   /* FDFS_FILE_EXT_NAME_MAX_LEN + 1 */

/* storage_gen_filename for a batch (storage/storage_service.c:2145-2202): the
 * 20-byte id le32(server_id) || be32(timestamp) || be64(masked size) ||
 * be32(crc32) in FastDFS base64 (A-Z a-z 0-9 - _, no padding) -> 27 chars per
 * file in name_out (no NUL).  masked size = COMBINE_RAND_FILE_SIZE (:2136)
 * with the caller's rand() draw rnd[i] when the size is below 2^32, else the
 * size (callers set the trunk / appender marks in file_size).  sub_path_out
 * [2i], [2i+1] = sub_path_high / low of storage_get_store_path's random mode
 * (:2128-2132): n = PJWHash(name) % 65536, (n >> 8) % subdir_count,
 * (n & 0xFF) % subdir_count; subdir_count in [1, 256].  The logical name is
 * "M%02d/%02X/%02X/" + name + ext, assembled by the caller.
 * Device arrays: crc32, file_size, timestamp, rnd [n]; name_out [n*27];
 * sub_path_out [n*2]. */
int fdfs_gpu_file_ids(fdfs_gpu_ctx *ctx, uint32_t server_id, const uint32_t *crc32,
                      const int64_t *file_size, const int32_t *timestamp, const uint32_t *rnd,
                      uint32_t n, uint32_t subdir_count, char *name_out, uint8_t *sub_path_out,
                      void *stream);

/* Decode of the 27-char name core as fdfs_get_file_info_ex does
 * (client/storage_client.c:2133-2214): server id, create timestamp, crc32 and
 * the file size under the master-file rule (low 32 bits when the size was
 * masked or carries the trunk mark, -1 for an appender file).  Slave names
 * (detected there by the full name length) are the caller's to flag. */
int fdfs_gpu_parse_file_ids(fdfs_gpu_ctx *ctx, const char *names, uint32_t n,
                            uint32_t *server_id_out, int32_t *timestamp_out,
                            int64_t *file_size_out, uint32_t *crc32_out, void *stream);

/* trunk_pack_header / trunk_unpack_header (storage/trunk_mgr/trunk_shared.c:
 * 340-370), 24 bytes per file: type, be32 alloc_size, be32 file_size,
 * be32 crc32, be32 mtime, 7-byte formatted ext name (ext: n*7 bytes). */
int fdfs_gpu_trunk_pack(fdfs_gpu_ctx *ctx, const uint8_t *file_type, const int32_t *alloc_size,
                        const int32_t *file_size, const uint32_t *crc32, const int32_t *mtime,
                        const char *ext, uint32_t n, uint8_t *hdr_out, void *stream);
int fdfs_gpu_trunk_unpack(fdfs_gpu_ctx *ctx, const uint8_t *hdr, uint32_t n, uint8_t *file_type,
                          int32_t *alloc_size, int32_t *file_size, uint32_t *crc32,
                          int32_t *mtime, char *ext, void *stream);

/* FastDHT routing of the dedup keys (ns, sig, "fid") for a batch: key_hash =
 * PJWHash(ns || 0x01 || sig) (CALC_KEY_HASH_CODE, storage/fdht_client/
 * fdht_client.c:256-305), group = key_hash % group_count (:375-376), server =
 * index inside the group from get_connection's rotate-16 (:207-212;
 * servers_per_group: device uint32[group_count], or NULL for 1 each).
 * order_out (device uint64[n], optional) lists the records group by group
 * (order inside a group unspecified) and group_start_out (device
 * uint64[group_count+1]) the group boundaries: one fdht_batch_set_ex (:512)
 * per group instead of one RPC per file.  ns: host string, 1..64 bytes. */
int fdfs_gpu_fdht_route(fdfs_gpu_ctx *ctx, const uint8_t *sig, uint64_t n, const char *ns,
                        int ns_len, uint32_t group_count, const uint32_t *servers_per_group,
                        int32_t *key_hash_out, uint32_t *group_out, uint32_t *server_out,
                        uint64_t *order_out, uint64_t *group_start_out, void *stream);

/* The same routing for any FastDHT object ids: `n` records of `key_stride`
 * bytes (4-aligned device buffer, key_stride a multiple of 4 and <= 128 =
 * FDHT_MAX_OBJECT_ID_LEN), the first key_len[i] bytes of record i hashed
 * (key_len: device uint32[n], or NULL for key_stride bytes each).  The "ref"
 * and "sig" keys of storage_set_link_file_meta (storage/storage_service.c:
 * 2948-3020) use the file id string ("group/M00/00/00/..ext") as object id.
 * fdfs_gpu_fdht_route is this call with 24-byte signature records. */
int fdfs_gpu_fdht_route_keys(fdfs_gpu_ctx *ctx, const uint8_t *keys, uint32_t key_stride,
                             const uint32_t *key_len, uint64_t n, const char *ns, int ns_len,
                             uint32_t group_count, const uint32_t *servers_per_group,
                             int32_t *key_hash_out, uint32_t *group_out, uint32_t *server_out,
                             uint64_t *order_out, uint64_t *group_start_out, void *stream);

/* ---- Recovery / sync-receiver batch ----------------------
 * Files that already carry their file ids (storage_disk_recovery,
 * storage/storage_disk_recovery.c:512-761; the sync receiver,
 * storage/storage_service.c:5468-5779) get in one stream-ordered call what a
 * sequential ingest with check_file_duplicate leaves in FastDHT
 * (storage/storage_service.c:2616-2785, 2948-3020):
 *   crc / sig     CRC32 and 24-byte signature (fdfs_gpu_sig_batch, method
 *                 FDFS_SIG_HASH or FDFS_SIG_MD5)
 *   rep / ref     class source (first file of the batch with the signature)
 *                 and class size (fdfs_gpu_dedup)
 *   fid           key (ns, sig, "fid") -> file_ids[index] of the source;
 *                 one record per class, the first *nsources entries
 *   ref_rec       key (ns, source file id, "ref") -> class size; as fid
 *   sig_rec       key (ns, file id, "sig") -> sig; one record per file
 * each routed as fdfs_gpu_fdht_route_keys does (key hash, group, server,
 * records ordered group by group).  file_ids: n records of id_stride bytes
 * (4-aligned, <= 128), id_len[i] (device, or NULL) bytes of each. */
typedef struct {
    uint64_t *index;        /* [n] file of each record */
    int32_t *key_hash;      /* [n] */
    uint32_t *group;        /* [n] */
    uint32_t *server;       /* [n] */
    uint64_t *order;        /* [n] records group by group, or NULL */
    uint64_t *group_start;  /* [group_count + 1] */
} fdfs_gpu_routed;

typedef struct {
    uint32_t *crc;          /* [n] */
    uint8_t *sig;           /* [n * 24], 8-aligned */
    uint64_t *rep;          /* [n] */
    uint32_t *ref;          /* [n] */
    uint64_t *nsources;     /* device uint64: records in fid / ref_rec */
    fdfs_gpu_routed fid, ref_rec, sig_rec;
} fdfs_gpu_recovery_out;

int fdfs_gpu_recovery_batch(fdfs_gpu_ctx *ctx, const fdfs_gpu_batch *batch, int method,
                            const uint8_t *file_ids, uint32_t id_stride, const uint32_t *id_len,
                            const char *ns, int ns_len, uint32_t group_count,
                            const uint32_t *servers_per_group, fdfs_gpu_recovery_out *out,
                            void *stream);

/* Scrub: recompute the CRC32 of every file of the batch (as
 * FDFS_SIG_CRC_ONLY) and compare with expected_crc (e.g. from
 * fdfs_gpu_parse_file_ids): crc_out[n], bad_out[n] (1 = mismatch), nbad_out
 * (device uint32, mismatch count). */
int fdfs_gpu_scrub(fdfs_gpu_ctx *ctx, const fdfs_gpu_batch *batch, const uint32_t *expected_crc,
                   uint32_t *crc_out, uint8_t *bad_out, uint32_t *nbad_out, void *stream);

/* Last HIP error string of this context (for logging), never NULL. */
const char *fdfs_gpu_last_error(fdfs_gpu_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif
