/*
 * fdfs_crc32_gpu -- drop-in for client/fdfs_crc32.c on libfdfs_gpu.
 *
 * Same usage, output ("%u\n" of CRC32_FINAL(CRC32_ex(...)),
 * client/fdfs_crc32.c:97-101) and error convention (message + errno exit
 * status, client/fdfs_crc32.c:37-45).  Several files may be given: one CRC
 * per line, in argument order.  A leading -u selects the logical-shift
 * (zlib) variant; the default is the signed-int CRC32_ex libfastcommon
 * declares.  No environment variable changes a result.
 *
 * Like the reference, which reads each file in 512 KiB chunks and carries
 * the CRC32_ex value from chunk to chunk (client/fdfs_crc32.c:70-93), the
 * files are streamed: windows of at most FDFS_CRC32_WINDOW bytes are read
 * into one of two pinned buffers while the other crosses PCIe and is hashed,
 * and every file's running state lives on the device
 * (fdfs_gpu_update_batch / fdfs_gpu_final_batch).  Host memory stays at two
 * windows whatever the file sizes.
 */
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "../../include/fdfs_gpu.h"

#define FDFS_CRC32_WINDOW (64u << 20)
#define MAX_PIECES 65536u

static int fail_io(const char *what, const char *fn, int line, int e)
{
    printf("file: " __FILE__ ", line: %d, %s file %s fail, errno: %d, error info: %s\n", line, what,
           fn, e, strerror(e));
    return e;
}

static int read_exact(int fd, unsigned char *dst, size_t len)
{
    size_t done = 0;
    while (done < len) {
        ssize_t r = read(fd, dst + done, len - done);
        if (r <= 0)
            return r < 0 ? (errno ? errno : EIO) : EIO;
        done += (size_t)r;
    }
    return 0;
}

struct slot {
    unsigned char *host;   /* pinned window bytes */
    uint64_t *h_meta;      /* pinned: offsets[MAX_PIECES], sizes[MAX_PIECES], idx (u32) */
    void *dev;             /* device window bytes + metadata */
    hipEvent_t done;
    int used;
};

int main(int argc, char *argv[])
{
    int unsigned_hash = 0;
    if (argc >= 2 && strcmp(argv[1], "-u") == 0) {
        unsigned_hash = 1;
        argv++;
        argc--;
    }
    if (argc < 2) {
        printf("Usage: %s [-u] <filename> [filename ...]\n", argv[0]);
        return 1;
    }
    const uint32_t n = (uint32_t)(argc - 1);
    uint64_t *sizes = calloc(n, sizeof(uint64_t));
    uint32_t *crc = calloc(n, sizeof(uint32_t));
    if (!sizes || !crc)
        return ENOMEM;
    for (uint32_t i = 0; i < n; i++) {
        struct stat st;
        if (stat(argv[i + 1], &st) != 0)
            return fail_io("open", argv[i + 1], __LINE__, errno ? errno : EACCES);
        sizes[i] = (uint64_t)st.st_size;
    }
    /* the device first: without a GPU this fails loudly (ENODEV), there is
     * no CPU path */
    fdfs_gpu_ctx *ctx = NULL;
    int rc = fdfs_gpu_open(0, unsigned_hash ? FDFS_GPU_FLAG_UNSIGNED_HASH : 0, &ctx);
    if (rc) {
        printf("fdfs_gpu_open fail, errno: %d, error info: %s\n", rc, strerror(rc));
        return rc;
    }
    const size_t meta_bytes = (size_t)MAX_PIECES * (8 + 8 + 4);
    fdfs_gpu_file_state *states = NULL;
    uint32_t *d_crc = NULL;
    hipStream_t s = NULL;
    struct slot sl[2];
    memset(sl, 0, sizeof(sl));
    if (hipMalloc((void **)&states, (size_t)n * sizeof(fdfs_gpu_file_state)) != hipSuccess ||
        hipMalloc((void **)&d_crc, (size_t)n * 4) != hipSuccess ||
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        printf("device allocation fail, errno: %d, error info: %s\n", ENOMEM, strerror(ENOMEM));
        return ENOMEM;
    }
    for (int k = 0; k < 2; k++) {
        if (hipHostMalloc((void **)&sl[k].host, FDFS_CRC32_WINDOW, 0) != hipSuccess ||
            hipHostMalloc((void **)&sl[k].h_meta, meta_bytes, 0) != hipSuccess ||
            hipMalloc(&sl[k].dev, FDFS_CRC32_WINDOW + meta_bytes) != hipSuccess ||
            hipEventCreateWithFlags(&sl[k].done, hipEventDisableTiming) != hipSuccess) {
            printf("buffer allocation fail, errno: %d, error info: %s\n", ENOMEM, strerror(ENOMEM));
            return ENOMEM;
        }
    }
    if ((rc = fdfs_gpu_state_init(ctx, states, n, s)) != 0)
        goto gpu_fail;

    uint32_t i = 0;      /* current file */
    uint64_t a = 0;      /* bytes of it already read */
    int fd = -1;
    for (int k = 0; i < n; k ^= 1) {
        struct slot *w = &sl[k];
        if (w->used && hipEventSynchronize(w->done) != hipSuccess) {
            rc = EIO;
            goto gpu_fail;
        }
        uint64_t *offs = w->h_meta, *lens = offs + MAX_PIECES;
        uint32_t *idx = (uint32_t *)(lens + MAX_PIECES);
        uint64_t fill = 0;
        uint32_t m = 0;
        /* the window: consecutive files, at most one piece of each */
        while (i < n && m < MAX_PIECES && fill < FDFS_CRC32_WINDOW) {
            if (sizes[i] == 0) {
                i++;
                continue;
            }
            if (fd < 0 && (fd = open(argv[i + 1], O_RDONLY)) < 0)
                return fail_io("open", argv[i + 1], __LINE__, errno ? errno : EACCES);
            uint64_t take = sizes[i] - a;
            if (take > FDFS_CRC32_WINDOW - fill)
                take = FDFS_CRC32_WINDOW - fill;
            int e = read_exact(fd, w->host + fill, (size_t)take);
            if (e)
                return fail_io("read", argv[i + 1], __LINE__, e);
            offs[m] = fill;
            lens[m] = take;
            idx[m] = i;
            m++;
            fill += take;
            a += take;
            if (a < sizes[i])
                break; /* window full; the file continues in the next one */
            close(fd);
            fd = -1;
            i++;
            a = 0;
        }
        if (m == 0)
            break;
        unsigned char *d_data = (unsigned char *)w->dev;
        char *d_meta = (char *)w->dev + FDFS_CRC32_WINDOW;
        if (hipMemcpyAsync(d_data, w->host, fill, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipMemcpyAsync(d_meta, w->h_meta, meta_bytes, hipMemcpyHostToDevice, s) != hipSuccess) {
            rc = EIO;
            goto gpu_fail;
        }
        /* CRC32_ex(chunk, crc) for every file of the window
         * (client/fdfs_crc32.c:91), on the device */
        fdfs_gpu_batch b = {d_data, (const uint64_t *)d_meta, (const uint64_t *)(d_meta + 8u * MAX_PIECES), m};
        if ((rc = fdfs_gpu_update_batch(ctx, &b, (const uint32_t *)(d_meta + 16u * MAX_PIECES), FDFS_SIG_CRC_ONLY,
                                        states, s)) != 0)
            goto gpu_fail;
        if (hipEventRecord(w->done, s) != hipSuccess) {
            rc = EIO;
            goto gpu_fail;
        }
        w->used = 1;
    }
    /* CRC32_FINAL (client/fdfs_crc32.c:99) */
    if ((rc = fdfs_gpu_final_batch(ctx, states, NULL, n, FDFS_SIG_CRC_ONLY, d_crc, NULL, NULL, s)) != 0)
        goto gpu_fail;
    if (hipMemcpyAsync(crc, d_crc, (size_t)n * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        rc = EIO;
        goto gpu_fail;
    }
    for (uint32_t j = 0; j < n; j++)
        printf("%u\n", crc[j]);
    fdfs_gpu_close(ctx);
    return 0;

gpu_fail:
    printf("libfdfs_gpu fail, errno: %d, error info: %s (%s)\n", rc, strerror(rc), fdfs_gpu_last_error(ctx));
    return rc;
}
