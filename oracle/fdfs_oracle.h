/*
 * fdfs_oracle.h -- CPU restatement of FastDFS's upload-path CRC32 / dedup
 * signature arithmetic.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline.  The product
 * (libfdfs_gpu) never links or calls it.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - MD5: pinned by the RFC 1321 appendix A.5 test suite (tests/golden).
 *   - CRC32 "unsigned" variant: pinned by zlib.crc32 (tests/golden).
 *   - CRC32_ex / ELFHash_ex / simple_hash_ex / Time33Hash_ex as compiled in
 *     libfastcommon (signed-int variant, the default here): PARITY UNPINNED.
 *     libfastcommon (>= 1.0.24, fastdfs.spec:19) is not vendored in
 *     /root/reference and no reference test pins any value; the semantics are
 *     restated from the reference's own types (int crc32 at
 *     storage/storage_nio.h:95, client/fdfs_crc32.c:27) and HISTORY:541.
 *     Both shift semantics are implemented and selectable.
 */
#ifndef FDFS_ORACLE_H
#define FDFS_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* variant: 0 = signed int state, arithmetic >> (libfastcommon as declared);
 *          1 = unsigned state, logical >> (== zlib for CRC32). */
#define ORC_VARIANT_SIGNED   0
#define ORC_VARIANT_UNSIGNED 1

#define ORC_METHOD_CRC_ONLY 0
#define ORC_METHOD_HASH     1   /* STORAGE_FILE_SIGNATURE_METHOD_HASH, storage/storage_global.h:41 */
#define ORC_METHOD_MD5      2   /* STORAGE_FILE_SIGNATURE_METHOD_MD5,  storage/storage_global.h:42 */

#define ORC_CRC32_XINIT 0xFFFFFFFFu

typedef struct {
    uint32_t state[4];
    uint64_t count;          /* bytes fed so far */
    uint8_t  buffer[64];
} orc_md5_ctx;

uint32_t orc_crc_table_entry(int i);
int32_t orc_crc32_ex(const void *buf, size_t len, int32_t init, int variant);
int32_t orc_crc32_final(int32_t crc);
int32_t orc_elf_ex(const void *buf, size_t len, int32_t init, int variant);
int32_t orc_simple_ex(const void *buf, size_t len, int32_t init);
int32_t orc_time33_ex(const void *buf, size_t len, int32_t init);

void orc_hash4_init(int32_t h[4]);
void orc_hash4_calc(const void *buf, size_t len, int32_t h[4], int variant);
void orc_hash4_finish(int32_t h[4]);

void orc_md5_init(orc_md5_ctx *ctx);
void orc_md5_update(orc_md5_ctx *ctx, const void *buf, size_t len);
void orc_md5_final(uint8_t digest[16], orc_md5_ctx *ctx);

void orc_sig_pack(int64_t file_size, int method, const int32_t codes[4],
                  uint8_t sig[24]);

/* One file through the storage_write_to_file / dio_write_file sequence,
 * fed in chunks of `chunk` bytes.  crc_out = final CRC32 of the file;
 * sig_out (24 B) filled when method != CRC_ONLY; codes_out (4 x int32,
 * may be NULL) = file_hash_codes (the raw MD5 digest for METHOD_MD5). */
void orc_dio_file(const uint8_t *buf, size_t len, size_t chunk, int method,
                  int variant, uint32_t *crc_out, uint8_t *sig_out,
                  int32_t *codes_out);

/* Batch of files (offset/size into base), one thread per file over
 * `nthreads` pthreads.  Returns 0. */
int orc_dio_batch(const uint8_t *base, const uint64_t *offset,
                  const uint64_t *size, uint64_t n, size_t chunk, int method,
                  int variant, uint32_t *crc_out, uint8_t *sig_out,
                  int nthreads);

/* test/gen_files.c corpus: writes the 6 files back to back into out
 * (116,653,056 bytes) using glibc srand/rand. */
uint64_t orc_gen_files_total(void);
void orc_gen_files(uint8_t *out);

/* Bulk equivalent of the upload-done dedup decision
 * (storage/storage_service.c:2616-2785, :2984): files in ingest order;
 * rep_out[i] = index of the first file with sig[i] (the FastDHT "fid"
 * source), ref_out[i] = number of files sharing sig[i]. */
int orc_dedup(const uint8_t *sig, uint64_t n, uint64_t *rep_out,
              uint32_t *ref_out);


/* ---- formats that consume the CRC, FastDHT routing ------- */

/* PJWHash (libfastcommon hash.c, called at storage/storage_service.c:2130 and
 * storage/fdht_client/fdht_client.c:301): h = (h << 4) + b; if the top nibble
 * x is set, h = (h ^ (x >> 24)) & 0x0FFFFFFF; `x >> 24` arithmetic for the
 * signed-int state (variant 0).  PARITY UNPINNED (libfastcommon absent). */
int32_t orc_pjw_hash(const void *buf, size_t len, int variant);

/* FastDFS base64 (base64_init_ex(ctx, 0, '-', '_', '.'),
 * storage/trunk_mgr/trunk_shared.c:32): alphabet A-Z a-z 0-9 - _, no
 * padding (bPad = false at storage/storage_service.c:2176).  Returns the
 * encoded / decoded length. */
int orc_base64_encode(const uint8_t *src, int len, char *dst);
int orc_base64_decode(const char *src, int len, uint8_t *dst);

/* storage_gen_filename core (storage/storage_service.c:2145-2202):
 * buff = le32 server_id || be32 timestamp || be64 masked size || be32 crc32
 * (masked size = COMBINE_RAND_FILE_SIZE, :2136-2142, with rand() draw rnd,
 * when size < 2^32); name = 27-char base64 of buff; sub_path = the random
 * distribution of storage_get_store_path (:2128-2132). */
void orc_file_id(uint32_t server_id, int32_t timestamp, int64_t file_size,
                 uint32_t crc32, uint32_t rnd, int subdir_count, int variant,
                 char name[27], uint8_t sub_path[2]);
/* fdfs_get_file_info_ex's decode (client/storage_client.c:2133-2214) of a
 * 27-char name: server id, timestamp, the file size under the master-file
 * rule (low 32 bits for masked or trunk sizes, -1 for an appender), crc32. */
void orc_parse_file_id(const char name[27], uint32_t *server_id, int32_t *timestamp,
                       int64_t *file_size, uint32_t *crc32);

/* trunk_pack_header / trunk_unpack_header (storage/trunk_mgr/trunk_shared.c:
 * 340-370): 24 bytes = type, be32 alloc_size, be32 file_size, be32 crc32,
 * be32 mtime, 7 bytes formatted ext name. */
void orc_trunk_pack(uint8_t file_type, int32_t alloc_size, int32_t file_size,
                    uint32_t crc32, int32_t mtime, const char ext[7], uint8_t hdr[24]);

/* FastDHT routing of the dedup key (ns, sig24, "fid"):
 * CALC_KEY_HASH_CODE (storage/fdht_client/fdht_client.c:256-305) over
 * ns || 0x01 || sig, group = (unsigned)hash % group_count (:375-376), server
 * index in the group = get_connection's rotate-16 % count (:207-212). */
void orc_fdht_route(const char *ns, int ns_len, const uint8_t sig[24], uint32_t group_count,
                    uint32_t servers, int variant, int32_t *key_hash, uint32_t *group,
                    uint32_t *server);
/* The same for any object id (ns || 0x01 || obj, obj_len <= 128). */
void orc_fdht_route_key(const char *ns, int ns_len, const uint8_t *obj, int obj_len,
                        uint32_t group_count, uint32_t servers, int variant, int32_t *key_hash,
                        uint32_t *group, uint32_t *server);

/* orc_dedup's answers on nthreads host threads (hash partition, sort per
 * partition); the CPU dedup baseline. */
int orc_dedup_mt(const uint8_t *sig, uint64_t n, uint64_t *rep_out, uint32_t *ref_out, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
