/*
 * fdfs_crc32_gpu -- drop-in for client/fdfs_crc32.c on libfdfs_gpu.
 *
 * Same usage, output ("%u\n" of CRC32_FINAL(CRC32_ex(...)),
 * client/fdfs_crc32.c:97-101) and error convention (message + errno exit
 * status, client/fdfs_crc32.c:37-45).  Several files may be given: they are
 * hashed as one GPU batch and printed one CRC per line, in argument order.
 * Set FDFS_UNSIGNED_HASH=1 in the environment for the logical-shift variant.
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

static int read_all(const char *fn, unsigned char *dst, size_t len)
{
    int fd = open(fn, O_RDONLY);
    if (fd < 0)
        return errno ? errno : EACCES;
    size_t done = 0;
    while (done < len) {
        ssize_t r = read(fd, dst + done, len - done > (1u << 30) ? (1u << 30) : len - done);
        if (r <= 0) {
            int e = r < 0 ? errno : EIO;
            close(fd);
            return e ? e : EIO;
        }
        done += (size_t)r;
    }
    close(fd);
    return 0;
}

int main(int argc, char *argv[])
{
    if (argc < 2) {
        printf("Usage: %s <filename> [filename ...]\n", argv[0]);
        return 1;
    }
    const int n = argc - 1;
    uint64_t *offs = calloc((size_t)n, sizeof(uint64_t));
    uint64_t *sizes = calloc((size_t)n, sizeof(uint64_t));
    uint32_t *crc = calloc((size_t)n, sizeof(uint32_t));
    if (!offs || !sizes || !crc)
        return ENOMEM;
    uint64_t total = 0;
    for (int i = 0; i < n; i++) {
        struct stat st;
        if (stat(argv[i + 1], &st) != 0) {
            int e = errno ? errno : EACCES;
            printf("file: " __FILE__ ", line: %d, open file %s fail, errno: %d, error info: %s\n",
                   __LINE__, argv[i + 1], e, strerror(e));
            return e;
        }
        offs[i] = total;
        sizes[i] = (uint64_t)st.st_size;
        total += (sizes[i] + 15) & ~15ull;  /* 16-byte aligned file starts */
    }
    /* the device first: without a GPU this fails loudly (ENODEV), there is
     * no CPU path */
    const char *u = getenv("FDFS_UNSIGNED_HASH");
    fdfs_gpu_ctx *ctx = NULL;
    int rc = fdfs_gpu_open(0, (u && *u == '1') ? FDFS_GPU_FLAG_UNSIGNED_HASH : 0, &ctx);
    if (rc) {
        printf("fdfs_gpu_open fail, errno: %d, error info: %s\n", rc, strerror(rc));
        return rc;
    }
    unsigned char *host = NULL;
    if (hipHostMalloc((void **)&host, total ? total : 16, 0) != hipSuccess)
        return ENOMEM;
    for (int i = 0; i < n; i++) {
        int e = read_all(argv[i + 1], host + offs[i], (size_t)sizes[i]);
        if (e) {
            printf("file: " __FILE__ ", line: %d, read file %s fail, errno: %d, error info: %s\n",
                   __LINE__, argv[i + 1], e, strerror(e));
            return e;
        }
    }
    /* streamed to the device and hashed there (fdfs_gpu_sig_batch_host) */
    fdfs_gpu_batch b = {host, offs, sizes, (uint32_t)n};
    rc = fdfs_gpu_sig_batch_host(ctx, &b, FDFS_SIG_CRC_ONLY, crc, NULL, NULL, 0);
    if (rc) {
        printf("fdfs_gpu_sig_batch_host fail, errno: %d, error info: %s (%s)\n", rc, strerror(rc),
               fdfs_gpu_last_error(ctx));
        return rc;
    }
    for (int i = 0; i < n; i++)
        printf("%u\n", crc[i]);
    fdfs_gpu_close(ctx);
    return 0;
}
