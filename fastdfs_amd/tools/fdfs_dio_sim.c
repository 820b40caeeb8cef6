/*
 * fdfs_dio_sim -- the storage daemon's upload hashing loop on libfdfs_gpu.
 *
 * A disk-I/O thread of fdfs_storaged hashes each upload one received chunk
 * at a time: storage_write_to_file initialises the StorageFileContext values
 * (storage/storage_service.c:7147-7161), dio_write_file advances them by the
 * chunk just written (CRC32_ex, CALC_HASH_CODES4 or my_md5_update,
 * storage/storage_dio.c:465-483) and finalises them after the last chunk
 * (:498-515; STORAGE_GEN_FILE_SIGNATURE, storage/storage_service.c:106-120).
 * A connection's next chunk is only received after this one is written
 * (storage/storage_nio.c:466), so each wakeup of the thread has at most one
 * chunk per upload in flight.
 *
 * This program is that loop in the batched form INTEGRATION.md section 3
 * describes, written against include/fdfs_gpu.h alone: every file given is
 * one upload, at most -j uploads are in flight at once, and each wakeup
 * advances every in-flight upload by its next chunk in one
 * fdfs_gpu_update_batch call, then finalises the uploads that ended in one
 * fdfs_gpu_final_batch call.  Chunks are <= -c bytes (buff_size,
 * conf/storage.conf:52); an upload's first chunk is shorter by the -H header
 * bytes the first receive buffer also carries.  Chunks are read from the
 * files into one of two pinned buffers while the other wakeup's chunks cross
 * PCIe and are hashed.
 *
 * Output, one line per file in argument order: the CRC32 ("%u", as
 * fdfs_crc32 prints it), then for -m hash / -m md5 the 24-byte signature in
 * hex.  A summary goes to stderr.  Errors: message + errno exit status, as
 * client/fdfs_crc32.c does.  -u selects the logical-shift hash variant
 * (no environment variable changes a result).
 */
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "../../include/fdfs_gpu.h"

static int fail_io(const char *what, const char *fn, int line, int e)
{
    printf("file: " __FILE__ ", line: %d, %s file %s fail, errno: %d, error info: %s\n", line, what, fn, e,
           strerror(e));
    return e;
}

static int pread_exact(int fd, unsigned char *dst, size_t len, off_t at)
{
    size_t done = 0;
    while (done < len) {
        ssize_t r = pread(fd, dst + done, len - done, at + (off_t)done);
        if (r <= 0)
            return r < 0 ? (errno ? errno : EIO) : EIO;
        done += (size_t)r;
    }
    return 0;
}

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* One wakeup's buffers: chunk bytes, then the metadata of its m chunks
 * (offsets, sizes, state indices) and of the uploads it finalises. */
struct slot {
    unsigned char *host, *dev;
    hipEvent_t done;
    int used;
};

int main(int argc, char *argv[])
{
    int method = FDFS_SIG_HASH;
    uint64_t buff = 256u << 10; /* buff_size = 256KB, conf/storage.conf:52 */
    uint64_t hdr = 25;          /* proto header (10) + upload fields (15) in the first buffer */
    uint32_t jobs = 1024;
    int opt, unsigned_hash = 0;
    while ((opt = getopt(argc, argv, "um:c:H:j:")) != -1) {
        if (opt == 'm')
            method = !strcmp(optarg, "crc") ? FDFS_SIG_CRC_ONLY : !strcmp(optarg, "md5") ? FDFS_SIG_MD5 : FDFS_SIG_HASH;
        else if (opt == 'c')
            buff = strtoull(optarg, NULL, 10);
        else if (opt == 'H')
            hdr = strtoull(optarg, NULL, 10);
        else if (opt == 'j')
            jobs = (uint32_t)strtoul(optarg, NULL, 10);
        else if (opt == 'u')
            unsigned_hash = 1;
        else
            optind = argc + 1;
    }
    if (optind >= argc || buff == 0 || hdr >= buff || jobs == 0) {
        printf("Usage: %s [-u] [-m crc|hash|md5] [-c buff_size] [-H header_bytes] [-j uploads] <filename> ...\n",
               argv[0]);
        return 1;
    }
    const uint32_t n = (uint32_t)(argc - optind);
    char **names = argv + optind;
    uint64_t *sizes = calloc(n, sizeof(uint64_t)), *sent = calloc(n, sizeof(uint64_t));
    uint32_t *crc = calloc(n, sizeof(uint32_t)), *done_at = calloc(n, sizeof(uint32_t));
    unsigned char *sig = calloc((size_t)n, 24);
    int *fds = malloc(n * sizeof(int));
    if (!sizes || !sent || !crc || !done_at || !sig || !fds)
        return ENOMEM;
    for (uint32_t i = 0; i < n; i++) {
        struct stat st;
        if (stat(names[i], &st) != 0)
            return fail_io("open", names[i], __LINE__, errno ? errno : EACCES);
        sizes[i] = (uint64_t)st.st_size;
        fds[i] = -1;
    }
    if (jobs > n)
        jobs = n;

    /* the device first: without a GPU this fails loudly (ENODEV), there is
     * no CPU path */
    fdfs_gpu_ctx *ctx = NULL;
    int rc = fdfs_gpu_open(0, unsigned_hash ? FDFS_GPU_FLAG_UNSIGNED_HASH : 0, &ctx);
    if (rc) {
        printf("fdfs_gpu_open fail, errno: %d, error info: %s\n", rc, strerror(rc));
        return rc;
    }
    /* one state per upload (a daemon would recycle the slots of finished
     * uploads, initialising each with fdfs_gpu_state_init(ctx, states + slot, 1, s)) */
    const uint64_t data_bytes = (uint64_t)jobs * buff, meta_bytes = (uint64_t)jobs * (8 + 8 + 4 + 4);
    fdfs_gpu_file_state *states = NULL;
    uint32_t *d_crc = NULL;
    unsigned char *d_sig = NULL;
    hipStream_t s = NULL;
    struct slot sl[2];
    memset(sl, 0, sizeof(sl));
    if (hipMalloc((void **)&states, (size_t)n * sizeof(fdfs_gpu_file_state)) != hipSuccess ||
        hipMalloc((void **)&d_crc, (size_t)n * 4) != hipSuccess ||
        hipMalloc((void **)&d_sig, (size_t)n * 24) != hipSuccess ||
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        printf("device allocation fail, errno: %d, error info: %s\n", ENOMEM, strerror(ENOMEM));
        return ENOMEM;
    }
    for (int k = 0; k < 2; k++) {
        if (hipHostMalloc((void **)&sl[k].host, data_bytes + meta_bytes, 0) != hipSuccess ||
            hipMalloc((void **)&sl[k].dev, data_bytes + meta_bytes) != hipSuccess ||
            hipEventCreateWithFlags(&sl[k].done, hipEventDisableTiming) != hipSuccess) {
            printf("buffer allocation fail, errno: %d, error info: %s\n", ENOMEM, strerror(ENOMEM));
            return ENOMEM;
        }
    }
    if ((rc = fdfs_gpu_reserve(ctx, jobs, 0)) != 0 || (rc = fdfs_gpu_state_init(ctx, states, n, s)) != 0)
        goto gpu_fail;

    /* in flight: uploads [lo, hi) minus the finished ones, hi - lo <= jobs
     * live at once (the list `live` keeps them in arrival order) */
    uint32_t *live = malloc((size_t)jobs * sizeof(uint32_t));
    if (!live)
        return ENOMEM;
    uint32_t nlive = 0, next = 0, ndone = 0;
    uint64_t wakeups = 0, chunks = 0, bytes = 0;
    const double t0 = now_s();
    for (int k = 0; ndone < n; k ^= 1) {
        while (nlive < jobs && next < n) /* new connections fill the free places */
            live[nlive++] = next++;
        struct slot *w = &sl[k];
        if (w->used && hipEventSynchronize(w->done) != hipSuccess) {
            rc = EIO;
            goto gpu_fail;
        }
        uint64_t *offs = (uint64_t *)(w->host + data_bytes), *lens = offs + jobs;
        uint32_t *sidx = (uint32_t *)(lens + jobs), *fin = sidx + jobs;
        uint64_t fill = 0;
        uint32_t m = 0, nfin = 0, keep = 0;
        for (uint32_t q = 0; q < nlive; q++) { /* the next chunk of every live upload */
            const uint32_t i = live[q];
            const uint64_t cap = sent[i] == 0 ? buff - hdr : buff;
            const uint64_t take = sizes[i] - sent[i] < cap ? sizes[i] - sent[i] : cap;
            if (take) {
                if (fds[i] < 0 && (fds[i] = open(names[i], O_RDONLY)) < 0)
                    return fail_io("open", names[i], __LINE__, errno ? errno : EACCES);
                int e = pread_exact(fds[i], w->host + fill, (size_t)take, (off_t)sent[i]);
                if (e)
                    return fail_io("read", names[i], __LINE__, e);
                offs[m] = fill;
                lens[m] = take;
                sidx[m] = i;
                m++;
                fill += take;
                sent[i] += take;
            }
            if (sent[i] == sizes[i]) { /* last chunk (or an empty file): finalise this wakeup */
                fin[nfin++] = i;
                done_at[ndone + nfin - 1] = i;
                if (fds[i] >= 0)
                    close(fds[i]);
                fds[i] = -1;
            } else {
                live[keep++] = i;
            }
        }
        nlive = keep;
        unsigned char *d_data = w->dev;
        uint64_t *d_offs = (uint64_t *)(w->dev + data_bytes), *d_lens = d_offs + jobs;
        uint32_t *d_sidx = (uint32_t *)(d_lens + jobs), *d_fin = d_sidx + jobs;
        if ((fill && hipMemcpyAsync(d_data, w->host, fill, hipMemcpyHostToDevice, s) != hipSuccess) ||
            hipMemcpyAsync(d_offs, w->host + data_bytes, meta_bytes, hipMemcpyHostToDevice, s) != hipSuccess) {
            rc = EIO;
            goto gpu_fail;
        }
        fdfs_gpu_batch b = {d_data, d_offs, d_lens, m};
        if (m && (rc = fdfs_gpu_update_batch(ctx, &b, d_sidx, method, states, s)) != 0)
            goto gpu_fail;
        if (nfin && (rc = fdfs_gpu_final_batch(ctx, states, d_fin, nfin, method, d_crc + ndone,
                                               method == FDFS_SIG_CRC_ONLY ? NULL : d_sig + 24ull * ndone, NULL,
                                               s)) != 0)
            goto gpu_fail;
        if (hipEventRecord(w->done, s) != hipSuccess) {
            rc = EIO;
            goto gpu_fail;
        }
        w->used = 1;
        ndone += nfin;
        wakeups++;
        chunks += m;
        bytes += fill;
    }
    /* results in completion order, back to file order */
    uint32_t *h_crc = malloc((size_t)n * 4);
    unsigned char *h_sig = malloc((size_t)n * 24);
    if (!h_crc || !h_sig)
        return ENOMEM;
    if (hipMemcpyAsync(h_crc, d_crc, (size_t)n * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(h_sig, d_sig, (size_t)n * 24, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        rc = EIO;
        goto gpu_fail;
    }
    const double secs = now_s() - t0;
    for (uint32_t j = 0; j < n; j++) {
        crc[done_at[j]] = h_crc[j];
        memcpy(sig + 24ull * done_at[j], h_sig + 24ull * j, 24);
    }
    for (uint32_t i = 0; i < n; i++) {
        printf("%u", crc[i]);
        if (method != FDFS_SIG_CRC_ONLY) {
            putchar(' ');
            for (int q = 0; q < 24; q++)
                printf("%02x", sig[24ull * i + q]);
        }
        putchar('\n');
    }
    fprintf(stderr, "uploads %u, wakeups %llu, chunks %llu, bytes %llu, %.3f s, %.1f MB/s, %.1f us per wakeup\n", n,
            (unsigned long long)wakeups, (unsigned long long)chunks, (unsigned long long)bytes, secs,
            (double)bytes / secs / 1e6, 1e6 * secs / (double)(wakeups ? wakeups : 1));
    fdfs_gpu_close(ctx);
    return 0;

gpu_fail:
    printf("libfdfs_gpu fail, errno: %d, error info: %s (%s)\n", rc, strerror(rc), fdfs_gpu_last_error(ctx));
    return rc;
}
