/*
 * fdfs_oracle.c -- CPU restatement of the FastDFS upload-path CRC32 /
 * dedup-signature arithmetic.  TEST INFRASTRUCTURE ONLY (see header).
 *
 * The arithmetic lives in libfastcommon (hash.c / md5.c), which the
 * reference links with -lfastcommon (storage/Makefile.in:5,
 * client/Makefile.in:7) but does not vendor.  Each function below names the
 * reference call site whose behaviour it restates.  All integer arithmetic
 * is done on uint32_t with the shift semantics spelled out, so the C here
 * has no undefined or implementation-defined behaviour.
 */
#define _GNU_SOURCE
#include "fdfs_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ CRC32 */

static uint32_t g_crc_table[256];
static pthread_once_t g_crc_once = PTHREAD_ONCE_INIT;

/* Reflected CRC-32 table, polynomial 0xEDB88320 (libfastcommon hash.c
 * crc_table, the table CRC32_ex indexes). */
static void crc_table_build(void)
{
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++)
            c = (c & 1u) ? (0xEDB88320u ^ (c >> 1)) : (c >> 1);
        g_crc_table[i] = c;
    }
}

uint32_t orc_crc_table_entry(int i)
{
    pthread_once(&g_crc_once, crc_table_build);
    return g_crc_table[i & 0xFF];
}

/* x >> k on a signed 32-bit int as gcc compiles it (arithmetic). */
static inline uint32_t sar32(uint32_t x, int k)
{
    uint32_t r = x >> k;
    if (x & 0x80000000u)
        r |= ~(0xFFFFFFFFu >> k);
    return r;
}

/* CRC32_ex(key, key_len, init_value), called at storage/storage_dio.c:467
 * and client/fdfs_crc32.c:91:  int crc;  crc = crc_table[(crc ^ *p) & 0xFF]
 * ^ (crc >> 8);  -- with `int crc` the >> is arithmetic (variant SIGNED). */
int32_t orc_crc32_ex(const void *buf, size_t len, int32_t init, int variant)
{
    pthread_once(&g_crc_once, crc_table_build);
    const uint8_t *p = (const uint8_t *)buf;
    uint32_t c = (uint32_t)init;
    if (variant == ORC_VARIANT_SIGNED) {
        for (size_t i = 0; i < len; i++)
            c = g_crc_table[(c ^ p[i]) & 0xFFu] ^ sar32(c, 8);
    } else {
        for (size_t i = 0; i < len; i++)
            c = g_crc_table[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
    }
    return (int32_t)c;
}

/* CRC32_FINAL(crc) = crc ^ 0xFFFFFFFF: storage/storage_dio.c:500,
 * client/fdfs_crc32.c:99. */
int32_t orc_crc32_final(int32_t crc)
{
    return (int32_t)((uint32_t)crc ^ 0xFFFFFFFFu);
}

/* ----------------------------------------------------- the other 3 hashes */

/* ELFHash_ex, the h[1] of CALC_HASH_CODES4 (storage/storage_dio.c:475):
 *   h = (h << 4) + b;  if ((x = h & 0xF0000000) != 0) { h ^= x >> 24; h &= ~x; }
 * with int h, int x  -> x >> 24 arithmetic (variant SIGNED). */
int32_t orc_elf_ex(const void *buf, size_t len, int32_t init, int variant)
{
    const uint8_t *p = (const uint8_t *)buf;
    uint32_t h = (uint32_t)init;
    for (size_t i = 0; i < len; i++) {
        h = (h << 4) + p[i];
        uint32_t x = h & 0xF0000000u;
        if (x != 0) {
            h ^= (variant == ORC_VARIANT_SIGNED) ? sar32(x, 24) : (x >> 24);
            h &= ~x;
        }
    }
    return (int32_t)h;
}

/* simple_hash_ex, h[2] of CALC_HASH_CODES4: h = 31 * h + b (mod 2^32). */
int32_t orc_simple_ex(const void *buf, size_t len, int32_t init)
{
    const uint8_t *p = (const uint8_t *)buf;
    uint32_t h = (uint32_t)init;
    for (size_t i = 0; i < len; i++)
        h = 31u * h + p[i];
    return (int32_t)h;
}

/* Time33Hash_ex, h[3] of CALC_HASH_CODES4: h += (h << 5) + b (mod 2^32). */
int32_t orc_time33_ex(const void *buf, size_t len, int32_t init)
{
    const uint8_t *p = (const uint8_t *)buf;
    uint32_t h = (uint32_t)init;
    for (size_t i = 0; i < len; i++)
        h += (h << 5) + p[i];
    return (int32_t)h;
}

/* INIT_HASH_CODES4 (storage/storage_service.c:7156). */
void orc_hash4_init(int32_t h[4])
{
    h[0] = (int32_t)ORC_CRC32_XINIT;
    h[1] = 0;
    h[2] = 0;
    h[3] = 0;
}

/* CALC_HASH_CODES4 (storage/storage_dio.c:475): four separate byte passes. */
void orc_hash4_calc(const void *buf, size_t len, int32_t h[4], int variant)
{
    h[0] = orc_crc32_ex(buf, len, h[0], variant);
    h[1] = orc_elf_ex(buf, len, h[1], variant);
    h[2] = orc_simple_ex(buf, len, h[2]);
    h[3] = orc_time33_ex(buf, len, h[3]);
}

/* FINISH_HASH_CODES4 (storage/storage_dio.c:508): only h[0] is finalised. */
void orc_hash4_finish(int32_t h[4])
{
    h[0] = orc_crc32_final(h[0]);
}

/* -------------------------------------------------------------------- MD5 */
/* my_md5_init / my_md5_update / my_md5_final (storage/storage_service.c:7160,
 * storage/storage_dio.c:480,512): the RSA reference MD5 of RFC 1321,
 * restated here from the RFC's algorithm description (sections 3.1-3.5). */

static inline uint32_t rol32(uint32_t x, int s)
{
    return (x << s) | (x >> (32 - s));
}

static const uint32_t MD5_K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a,
    0xa8304613, 0xfd469501, 0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be,
    0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340,
    0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8,
    0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c,
    0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70, 0x289b7ec6, 0xeaa127fa,
    0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92,
    0xffeff47d, 0x85845dd1, 0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1,
    0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};

static const int MD5_S[64] = {
    7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
    5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
    4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
    6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static void md5_block(uint32_t st[4], const uint8_t blk[64])
{
    uint32_t m[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)blk[4 * i] | ((uint32_t)blk[4 * i + 1] << 8) |
               ((uint32_t)blk[4 * i + 2] << 16) |
               ((uint32_t)blk[4 * i + 3] << 24);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) {
            f = (b & c) | (~b & d);
            g = i;
        } else if (i < 32) {
            f = (d & b) | (~d & c);
            g = (5 * i + 1) & 15;
        } else if (i < 48) {
            f = b ^ c ^ d;
            g = (3 * i + 5) & 15;
        } else {
            f = c ^ (b | ~d);
            g = (7 * i) & 15;
        }
        uint32_t t = d;
        d = c;
        c = b;
        b = b + rol32(a + f + MD5_K[i] + m[g], MD5_S[i]);
        a = t;
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
}

void orc_md5_init(orc_md5_ctx *ctx)
{
    ctx->state[0] = 0x67452301u;
    ctx->state[1] = 0xefcdab89u;
    ctx->state[2] = 0x98badcfeu;
    ctx->state[3] = 0x10325476u;
    ctx->count = 0;
}

void orc_md5_update(orc_md5_ctx *ctx, const void *buf, size_t len)
{
    const uint8_t *p = (const uint8_t *)buf;
    size_t have = (size_t)(ctx->count & 63u);
    ctx->count += len;
    if (have) {
        size_t need = 64 - have;
        if (len < need) {
            memcpy(ctx->buffer + have, p, len);
            return;
        }
        memcpy(ctx->buffer + have, p, need);
        md5_block(ctx->state, ctx->buffer);
        p += need;
        len -= need;
    }
    while (len >= 64) {
        md5_block(ctx->state, p);
        p += 64;
        len -= 64;
    }
    if (len)
        memcpy(ctx->buffer, p, len);
}

void orc_md5_final(uint8_t digest[16], orc_md5_ctx *ctx)
{
    uint64_t bits = ctx->count * 8u;
    uint8_t pad[72];
    size_t have = (size_t)(ctx->count & 63u);
    size_t padlen = (have < 56) ? (56 - have) : (120 - have);
    memset(pad, 0, sizeof(pad));
    pad[0] = 0x80;
    uint8_t lenb[8];
    for (int i = 0; i < 8; i++)
        lenb[i] = (uint8_t)(bits >> (8 * i));
    uint64_t saved = ctx->count;
    orc_md5_update(ctx, pad, padlen);
    orc_md5_update(ctx, lenb, 8);
    ctx->count = saved;
    for (int i = 0; i < 4; i++)
        for (int k = 0; k < 4; k++)
            digest[4 * i + k] = (uint8_t)(ctx->state[i] >> (8 * k));
}

/* ------------------------------------------------------------- signature */

/* STORAGE_GEN_FILE_SIGNATURE (storage/storage_service.c:108-120):
 * long2buff(size) big-endian, then int2buff(h[i]) big-endian x4 for the
 * hash method, or the 16 raw digest bytes for MD5. */
void orc_sig_pack(int64_t file_size, int method, const int32_t codes[4],
                  uint8_t sig[24])
{
    uint64_t s = (uint64_t)file_size;
    for (int i = 0; i < 8; i++)
        sig[i] = (uint8_t)(s >> (56 - 8 * i));
    if (method == ORC_METHOD_HASH) {
        for (int k = 0; k < 4; k++) {
            uint32_t v = (uint32_t)codes[k];
            sig[8 + 4 * k] = (uint8_t)(v >> 24);
            sig[9 + 4 * k] = (uint8_t)(v >> 16);
            sig[10 + 4 * k] = (uint8_t)(v >> 8);
            sig[11 + 4 * k] = (uint8_t)v;
        }
    } else {
        memcpy(sig + 8, codes, 16);
    }
}

/* -------------------------------------------------------- dio file driver */

/* storage_write_to_file (storage/storage_service.c:7147-7161) initialises
 * the state, dio_write_file (storage/storage_dio.c:465-483) updates it once
 * per received chunk, and finalises after the last one (:498-515). */
void orc_dio_file(const uint8_t *buf, size_t len, size_t chunk, int method,
                  int variant, uint32_t *crc_out, uint8_t *sig_out,
                  int32_t *codes_out)
{
    int32_t crc = (int32_t)ORC_CRC32_XINIT;
    int32_t h[4];
    orc_md5_ctx md5;
    if (chunk == 0)
        chunk = len ? len : 1;
    if (method == ORC_METHOD_HASH)
        orc_hash4_init(h);
    else if (method == ORC_METHOD_MD5)
        orc_md5_init(&md5);

    for (size_t off = 0; off < len; off += chunk) {
        size_t n = (len - off < chunk) ? (len - off) : chunk;
        crc = orc_crc32_ex(buf + off, n, crc, variant);
        if (method == ORC_METHOD_HASH)
            orc_hash4_calc(buf + off, n, h, variant);
        else if (method == ORC_METHOD_MD5)
            orc_md5_update(&md5, buf + off, n);
    }
    crc = orc_crc32_final(crc);
    if (method == ORC_METHOD_HASH)
        orc_hash4_finish(h);
    else if (method == ORC_METHOD_MD5)
        orc_md5_final((uint8_t *)h, &md5);

    if (crc_out)
        *crc_out = (uint32_t)crc;
    if (method != ORC_METHOD_CRC_ONLY) {
        if (sig_out)
            orc_sig_pack((int64_t)len, method, h, sig_out);
        if (codes_out)
            memcpy(codes_out, h, 16);
    }
}

typedef struct {
    const uint8_t *base;
    const uint64_t *offset, *size;
    uint64_t n;
    size_t chunk;
    int method, variant;
    uint32_t *crc_out;
    uint8_t *sig_out;
    uint64_t next;  /* shared work counter */
} batch_job;

static void *batch_worker(void *arg)
{
    batch_job *j = (batch_job *)arg;
    for (;;) {
        uint64_t i = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (i >= j->n)
            break;
        orc_dio_file(j->base + j->offset[i], (size_t)j->size[i], j->chunk,
                     j->method, j->variant, j->crc_out ? j->crc_out + i : NULL,
                     j->sig_out ? j->sig_out + 24 * i : NULL, NULL);
    }
    return NULL;
}

int orc_dio_batch(const uint8_t *base, const uint64_t *offset,
                  const uint64_t *size, uint64_t n, size_t chunk, int method,
                  int variant, uint32_t *crc_out, uint8_t *sig_out,
                  int nthreads)
{
    batch_job j = {base, offset, size, n, chunk, method, variant,
                   crc_out, sig_out, 0};
    if (nthreads <= 1) {
        batch_worker(&j);
        return 0;
    }
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    if (!th)
        return 12;
    for (int t = 0; t < nthreads; t++)
        pthread_create(&th[t], NULL, batch_worker, &j);
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    free(th);
    return 0;
}

/* ------------------------------------------------------ gen_files corpus */

/* test/gen_files.c:14-21 sizes, test/test_types.h:19 seed. */
static const uint32_t GEN_SIZES[6] = {5 * 1024, 50 * 1024, 200 * 1024,
                                      1 * 1024 * 1024, 10 * 1024 * 1024,
                                      100 * 1024 * 1024};
#define GEN_SRAND_SEED 1225420780u
#define GEN_BLOCK 1024

uint64_t orc_gen_files_total(void)
{
    uint64_t t = 0;
    for (int i = 0; i < 6; i++)
        t += GEN_SIZES[i];
    return t;
}

/* test/gen_files.c:34,46-64: one glibc rand() stream across all six files;
 * each file is (bytes/1024 - 1) random 1 KiB blocks, byte =
 * (int)(255 * ((double)rand() / RAND_MAX)), then one 1 KiB block of 0xFF. */
void orc_gen_files(uint8_t *out)
{
    srand(GEN_SRAND_SEED);
    uint8_t *p = out;
    for (int f = 0; f < 6; f++) {
        int loop = (int)(GEN_SIZES[f] / GEN_BLOCK);
        for (int k = 0; k < loop - 1; k++)
            for (int b = 0; b < GEN_BLOCK; b++)
                *p++ = (uint8_t)(int)(255 * ((double)rand() / RAND_MAX));
        memset(p, 0xFF, GEN_BLOCK);
        p += GEN_BLOCK;
    }
}

/* ------------------------------------------------------------------ dedup */

static const uint8_t *g_sort_sig;

static int sig_idx_cmp(const void *a, const void *b)
{
    uint64_t ia = *(const uint64_t *)a, ib = *(const uint64_t *)b;
    int c = memcmp(g_sort_sig + 24 * ia, g_sort_sig + 24 * ib, 24);
    if (c)
        return c;
    return (ia > ib) - (ia < ib);
}

/* Sequential FastDHT semantics of storage_service_upload_file_done
 * (storage/storage_service.c:2652 get "fid": hit -> link to source;
 * :2714 miss -> this file becomes the source) and storage_set_link_file_meta
 * (:2984 fdht_inc "ref" +1 per link): after ingesting all n files in order,
 * every file links to the first file with its signature and the class's ref
 * equals its size.  Not thread-safe (qsort comparator global). */
int orc_dedup(const uint8_t *sig, uint64_t n, uint64_t *rep_out,
              uint32_t *ref_out)
{
    uint64_t *ord = (uint64_t *)malloc(sizeof(uint64_t) * (n ? n : 1));
    if (!ord)
        return 12;
    for (uint64_t i = 0; i < n; i++)
        ord[i] = i;
    g_sort_sig = sig;
    qsort(ord, (size_t)n, sizeof(uint64_t), sig_idx_cmp);
    uint64_t s = 0;
    while (s < n) {
        uint64_t e = s + 1;
        while (e < n && memcmp(sig + 24 * ord[s], sig + 24 * ord[e], 24) == 0)
            e++;
        for (uint64_t k = s; k < e; k++) {
            rep_out[ord[k]] = ord[s];
            ref_out[ord[k]] = (uint32_t)(e - s);
        }
        s = e;
    }
    free(ord);
    return 0;
}

/* The same answers on `nthreads` host threads (the multi-core CPU
 * baseline of bench.py): records are partitioned by a hash of
 * their 24 bytes (equal signatures share a partition, indices stay
 * ascending inside it), each partition is sorted by (signature, index) and
 * its runs are the classes.  Same output as orc_dedup. */
typedef struct {
    const uint8_t *sig;
    uint64_t n, *idx, *start, *tcount;
    uint32_t nb, nt;
    uint64_t *rep;
    uint32_t *ref;
    uint32_t next;  /* partition work counter */
    int phase;
    int tid_next;
} dd_job;

static inline uint32_t dd_bucket(const uint8_t *r, uint32_t nb)
{
    uint64_t a, b, c;
    memcpy(&a, r, 8);
    memcpy(&b, r + 8, 8);
    memcpy(&c, r + 16, 8);
    uint64_t h = (a * 0x9E3779B97F4A7C15ull) ^ (b * 0xC2B2AE3D27D4EB4Full) ^ (c * 0x165667B19E3779F9ull);
    h ^= h >> 29;
    return (uint32_t)((h * 0xBF58476D1CE4E5B9ull) >> 32) % nb;
}

static int dd_cmp(const void *x, const void *y, void *arg)
{
    const uint8_t *sig = (const uint8_t *)arg;
    const uint64_t ia = *(const uint64_t *)x, ib = *(const uint64_t *)y;
    const int c = memcmp(sig + 24 * ia, sig + 24 * ib, 24);
    return c ? c : (ia > ib) - (ia < ib);
}

static void *dd_worker(void *arg)
{
    dd_job *j = (dd_job *)arg;
    const uint32_t t = (uint32_t)__atomic_fetch_add(&j->tid_next, 1, __ATOMIC_RELAXED);
    const uint64_t lo = j->n * t / j->nt, hi = j->n * (t + 1) / j->nt;
    uint64_t *cnt = j->tcount + (uint64_t)t * j->nb;
    if (j->phase == 0) {  /* count this thread's slice per partition */
        for (uint64_t i = lo; i < hi; i++)
            cnt[dd_bucket(j->sig + 24 * i, j->nb)]++;
    } else if (j->phase == 1) {  /* scatter (cnt holds this slice's write cursors) */
        for (uint64_t i = lo; i < hi; i++)
            j->idx[cnt[dd_bucket(j->sig + 24 * i, j->nb)]++] = i;
    } else {  /* sort + group partitions */
        for (;;) {
            const uint32_t b = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
            if (b >= j->nb)
                break;
            uint64_t *o = j->idx + j->start[b];
            const uint64_t m = j->start[b + 1] - j->start[b];
            qsort_r(o, (size_t)m, sizeof(uint64_t), dd_cmp, (void *)j->sig);
            uint64_t s = 0;
            while (s < m) {
                uint64_t e = s + 1;
                while (e < m && memcmp(j->sig + 24 * o[s], j->sig + 24 * o[e], 24) == 0)
                    e++;
                for (uint64_t k = s; k < e; k++) {
                    j->rep[o[k]] = o[s];
                    j->ref[o[k]] = (uint32_t)(e - s);
                }
                s = e;
            }
        }
    }
    return NULL;
}

static void dd_run(dd_job *j)
{
    pthread_t th[256];
    j->tid_next = 0;
    for (uint32_t t = 0; t < j->nt; t++)
        pthread_create(&th[t], NULL, dd_worker, j);
    for (uint32_t t = 0; t < j->nt; t++)
        pthread_join(th[t], NULL);
}

int orc_dedup_mt(const uint8_t *sig, uint64_t n, uint64_t *rep_out, uint32_t *ref_out, int nthreads)
{
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    dd_job j;
    memset(&j, 0, sizeof(j));
    j.sig = sig;
    j.n = n;
    j.nt = (uint32_t)nthreads;
    /* partitions of ~2K records: each one's random signature reads stay in cache */
    uint64_t nb = n / 2048;
    if (nb < 64u * (uint64_t)nthreads)
        nb = 64u * (uint64_t)nthreads;
    if (nb > (1u << 20))
        nb = 1u << 20;
    j.nb = (uint32_t)nb;
    j.rep = rep_out;
    j.ref = ref_out;
    j.idx = (uint64_t *)malloc(sizeof(uint64_t) * (n ? n : 1));
    j.start = (uint64_t *)calloc(j.nb + 1, sizeof(uint64_t));
    j.tcount = (uint64_t *)calloc((size_t)j.nb * j.nt, sizeof(uint64_t));
    if (!j.idx || !j.start || !j.tcount) {
        free(j.idx);
        free(j.start);
        free(j.tcount);
        return 12;
    }
    j.phase = 0;
    dd_run(&j);
    /* partition starts, and each slice's cursor inside each partition
     * (slices in order, so indices stay ascending in a partition) */
    uint64_t run = 0;
    for (uint32_t b = 0; b < j.nb; b++) {
        j.start[b] = run;
        for (uint32_t t = 0; t < j.nt; t++) {
            const uint64_t c = j.tcount[(uint64_t)t * j.nb + b];
            j.tcount[(uint64_t)t * j.nb + b] = run;
            run += c;
        }
    }
    j.start[j.nb] = run;
    j.phase = 1;
    dd_run(&j);
    j.phase = 2;
    dd_run(&j);
    free(j.idx);
    free(j.start);
    free(j.tcount);
    return 0;
}

/* ---- formats that consume the CRC, FastDHT routing -------------------- */

int32_t orc_pjw_hash(const void *buf, size_t len, int variant)
{
    const uint8_t *p = (const uint8_t *)buf;
    uint32_t h = 0;
    for (size_t i = 0; i < len; i++) {
        h = (h << 4) + p[i];
        const uint32_t x = h & 0xF0000000u;
        if (x) {
            const uint32_t s = variant == ORC_VARIANT_SIGNED ? sar32(x, 24) : (x >> 24);
            h = (h ^ s) & 0x0FFFFFFFu;
        }
    }
    return (int32_t)h;
}

static const char B64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";

int orc_base64_encode(const uint8_t *src, int len, char *dst)
{
    int o = 0, i = 0;
    for (; i + 3 <= len; i += 3) {
        const uint32_t v = ((uint32_t)src[i] << 16) | ((uint32_t)src[i + 1] << 8) | src[i + 2];
        dst[o++] = B64[v >> 18];
        dst[o++] = B64[(v >> 12) & 63];
        dst[o++] = B64[(v >> 6) & 63];
        dst[o++] = B64[v & 63];
    }
    if (len - i == 1) {
        const uint32_t v = (uint32_t)src[i] << 16;
        dst[o++] = B64[v >> 18];
        dst[o++] = B64[(v >> 12) & 63];
    } else if (len - i == 2) {
        const uint32_t v = ((uint32_t)src[i] << 16) | ((uint32_t)src[i + 1] << 8);
        dst[o++] = B64[v >> 18];
        dst[o++] = B64[(v >> 12) & 63];
        dst[o++] = B64[(v >> 6) & 63];
    }
    return o;
}

static int b64_val(char c)
{
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '-') return 62;
    if (c == '_') return 63;
    return -1;
}

int orc_base64_decode(const char *src, int len, uint8_t *dst)
{
    uint32_t acc = 0;
    int bits = 0, o = 0;
    for (int i = 0; i < len; i++) {
        const int v = b64_val(src[i]);
        if (v < 0)
            break;  /* pad '.' or end */
        acc = (acc << 6) | (uint32_t)v;
        bits += 6;
        if (bits >= 8) {
            bits -= 8;
            dst[o++] = (uint8_t)(acc >> bits);
        }
    }
    return o;
}

static void put_be32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

static uint32_t get_be32(const uint8_t *p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

void orc_file_id(uint32_t server_id, int32_t timestamp, int64_t file_size,
                 uint32_t crc32, uint32_t rnd, int subdir_count, int variant,
                 char name[27], uint8_t sub_path[2])
{
    uint8_t buff[20];
    /* int2buff(htonl(id)) on a little-endian host: the id's LE bytes */
    buff[0] = (uint8_t)server_id; buff[1] = (uint8_t)(server_id >> 8);
    buff[2] = (uint8_t)(server_id >> 16); buff[3] = (uint8_t)(server_id >> 24);
    put_be32(buff + 4, (uint32_t)timestamp);
    uint64_t masked = (uint64_t)file_size;
    if ((file_size >> 32) == 0) {  /* COMBINE_RAND_FILE_SIZE */
        const uint32_t r = (rnd & 0x007FFFFFu) | 0x80000000u;
        masked = ((uint64_t)r << 32) | (uint64_t)file_size;
    }
    put_be32(buff + 8, (uint32_t)(masked >> 32));
    put_be32(buff + 12, (uint32_t)masked);
    put_be32(buff + 16, crc32);
    orc_base64_encode(buff, 20, name);
    const uint32_t h = (uint32_t)orc_pjw_hash(name, 27, variant) % (1u << 16);
    sub_path[0] = (uint8_t)(((h >> 8) & 0xFF) % (uint32_t)subdir_count);
    sub_path[1] = (uint8_t)((h & 0xFF) % (uint32_t)subdir_count);
}

void orc_parse_file_id(const char name[27], uint32_t *server_id, int32_t *timestamp,
                       int64_t *file_size, uint32_t *crc32)
{
    uint8_t buff[21];
    orc_base64_decode(name, 27, buff);
    *server_id = (uint32_t)buff[0] | ((uint32_t)buff[1] << 8) | ((uint32_t)buff[2] << 16) |
                 ((uint32_t)buff[3] << 24);
    *timestamp = (int32_t)get_be32(buff + 4);
    int64_t sz = (int64_t)(((uint64_t)get_be32(buff + 8) << 32) | get_be32(buff + 12));
    const int64_t kAppender = 1LL << 58, kTrunk = 1LL << 59;  /* INFINITE_FILE_SIZE, FDFS_TRUNK_FILE_MARK_SIZE */
    *crc32 = get_be32(buff + 16);
    if (sz & kAppender) {          /* IS_APPENDER_FILE: size -1, crc32 left 0 (:2181-2201) */
        sz = -1;
        *crc32 = 0;
    } else if ((uint64_t)sz >> 63) /* master file (:2203-2213) */
        sz &= 0xFFFFFFFFLL;
    else if (sz & kTrunk)
        sz &= 0xFFFFFFFFLL;        /* FDFS_TRUNK_FILE_TRUE_SIZE */
    *file_size = sz;
}

void orc_trunk_pack(uint8_t file_type, int32_t alloc_size, int32_t file_size,
                    uint32_t crc32, int32_t mtime, const char ext[7], uint8_t hdr[24])
{
    hdr[0] = file_type;
    put_be32(hdr + 1, (uint32_t)alloc_size);
    put_be32(hdr + 5, (uint32_t)file_size);
    put_be32(hdr + 9, crc32);
    put_be32(hdr + 13, (uint32_t)mtime);
    memcpy(hdr + 17, ext, 7);
}

void orc_fdht_route(const char *ns, int ns_len, const uint8_t sig[24], uint32_t group_count,
                    uint32_t servers, int variant, int32_t *key_hash, uint32_t *group,
                    uint32_t *server)
{
    orc_fdht_route_key(ns, ns_len, sig, 24, group_count, servers, variant, key_hash, group, server);
}

void orc_fdht_route_key(const char *ns, int ns_len, const uint8_t *obj, int obj_len,
                        uint32_t group_count, uint32_t servers, int variant, int32_t *key_hash,
                        uint32_t *group, uint32_t *server)
{
    uint8_t key[64 + 1 + 128];
    memcpy(key, ns, (size_t)ns_len);
    key[ns_len] = 0x01;  /* FDHT_FULL_KEY_SEPERATOR */
    memcpy(key + ns_len + 1, obj, (size_t)obj_len);
    int32_t h = orc_pjw_hash(key, (size_t)ns_len + 1 + (size_t)obj_len, variant);
    if (h < 0)
        h &= 0x7FFFFFFF;
    *key_hash = h;
    *group = (uint32_t)h % group_count;
    int32_t nh = (int32_t)(((uint32_t)h << 16) | ((uint32_t)h >> 16));
    if (nh < 0)
        nh &= 0x7FFFFFFF;
    *server = (uint32_t)nh % servers;
}
