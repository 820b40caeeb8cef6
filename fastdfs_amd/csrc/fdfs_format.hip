// libfdfs_gpu: the formats that consume the file CRC, and the FastDHT routing
// of the dedup keys, for whole batches.
//
//  * file_id_kernel: storage_gen_filename (storage/storage_service.c:
//    2145-2202): the 20-byte id (le32 server id, be32 timestamp, be64 masked
//    size, be32 crc32) in FastDFS base64 (27 chars), and the store sub path
//    of storage_get_store_path's random mode (:2128-2132, PJWHash of the
//    name).  One thread per file.
//  * parse_file_id_kernel: fdfs_get_file_info_ex's decode
//    (client/storage_client.c:2133-2214) -- the download / scrub side.
//  * trunk_pack_kernel / trunk_unpack_kernel: trunk_pack_header /
//    trunk_unpack_header (storage/trunk_mgr/trunk_shared.c:340-370).
//  * fdht_route_kernel + group counting sort: the FastDHT partition of the
//    dedup keys ((ns, sig, "fid"), (ns, file id, "ref" / "sig")): CALC_KEY_HASH_CODE
//    (storage/fdht_client/fdht_client.c:256-305), group = hash % group_count
//    (:375-376), server = get_connection's rotate-16 % count (:207-212), and
//    the records ordered by group so each group's keys go out in one
//    fdht_batch_set_ex (:512) instead of one RPC per file.
//  * scrub_kernel: compare recomputed CRCs with expected ones (download-side
//    verification; the CRCs come from crc_seg_kernel).
//
// All of it is a few bytes per record: HBM-bound byte work, no LDS.
#include "fdfs_device.hpp"
#include "fdfs_kernels.hpp"

namespace fdfs {

__device__ __forceinline__ char b64_char(uint32_t v)
{
    // A-Z a-z 0-9 - _  (base64_init_ex(ctx, 0, '-', '_', '.'), trunk_shared.c:32)
    return v < 26 ? (char)('A' + v) : v < 52 ? (char)('a' + v - 26) : v < 62 ? (char)('0' + v - 52)
                                                                      : (v == 62 ? '-' : '_');
}

__device__ __forceinline__ uint32_t b64_value(uint8_t c)
{
    return (c >= 'A' && c <= 'Z') ? c - 'A' : (c >= 'a' && c <= 'z') ? c - 'a' + 26
           : (c >= '0' && c <= '9') ? c - '0' + 52 : (c == '-' ? 62u : 63u);
}

// PJWHash (libfastcommon hash.c): h = (h << 4) + b; top nibble x folded in
// as (h ^ (x >> 24)) & 0x0FFFFFFF, `>>` arithmetic for the signed state.
template <bool SAR>
__device__ __forceinline__ uint32_t pjw_step(uint32_t h, uint32_t b)
{
    h = (h << 4) + b;
    const uint32_t x = h & 0xF0000000u;
    if (x)
        h = (h ^ (SAR ? (uint32_t)((int32_t)x >> 24) : (x >> 24))) & 0x0FFFFFFFu;
    return h;
}

template <bool SAR>
__global__ void file_id_kernel(uint32_t server_id, const uint32_t *__restrict__ crc32,
                               const int64_t *__restrict__ size, const int32_t *__restrict__ ts,
                               const uint32_t *__restrict__ rnd, uint32_t n, uint32_t subdirs,
                               char *__restrict__ name_out, uint8_t *__restrict__ sub_out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const int64_t L = size[i];
    uint64_t masked = (uint64_t)L;
    if ((L >> 32) == 0)  // COMBINE_RAND_FILE_SIZE (storage/storage_service.c:2136-2142)
        masked = ((uint64_t)((rnd[i] & 0x007FFFFFu) | 0x80000000u) << 32) | (uint64_t)L;
    uint8_t b[21];
    b[0] = (uint8_t)server_id;  // int2buff(htonl(id)): the id's little-endian bytes
    b[1] = (uint8_t)(server_id >> 8);
    b[2] = (uint8_t)(server_id >> 16);
    b[3] = (uint8_t)(server_id >> 24);
    const uint32_t w[4] = {(uint32_t)ts[i], (uint32_t)(masked >> 32), (uint32_t)masked, crc32[i]};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        b[4 + 4 * k] = (uint8_t)(w[k] >> 24);
        b[5 + 4 * k] = (uint8_t)(w[k] >> 16);
        b[6 + 4 * k] = (uint8_t)(w[k] >> 8);
        b[7 + 4 * k] = (uint8_t)w[k];
    }
    b[20] = 0;
    char name[28];
    uint32_t h = 0;
#pragma unroll
    for (int g = 0; g < 7; g++) {  // 6 full groups + 2 trailing bytes -> 27 chars
        const uint32_t v = ((uint32_t)b[3 * g] << 16) | ((uint32_t)b[3 * g + 1] << 8) |
                           (g < 6 ? b[3 * g + 2] : 0u);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (g == 6 && q == 3)
                break;
            const char ch = b64_char((v >> (18 - 6 * q)) & 63u);
            name[4 * g + q] = ch;
            h = pjw_step<SAR>(h, (uint8_t)ch);
        }
    }
    char *o = name_out + 27ull * i;
#pragma unroll
    for (int k = 0; k < 27; k++)
        o[k] = name[k];
    const uint32_t nn = h % (1u << 16);  // storage_get_store_path, random mode
    sub_out[2ull * i] = (uint8_t)(((nn >> 8) & 0xFFu) % subdirs);
    sub_out[2ull * i + 1] = (uint8_t)((nn & 0xFFu) % subdirs);
}

__global__ void parse_file_id_kernel(const uint8_t *__restrict__ names, uint32_t n,
                                     uint32_t *__restrict__ sid_out, int32_t *__restrict__ ts_out,
                                     int64_t *__restrict__ size_out, uint32_t *__restrict__ crc_out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint8_t *s = names + 27ull * i;
    uint8_t b[21];
#pragma unroll
    for (int g = 0; g < 7; g++) {
        uint32_t v = 0;
#pragma unroll
        for (int q = 0; q < 4; q++)
            v = (v << 6) | ((g == 6 && q == 3) ? 0u : b64_value(s[4 * g + q]));
        b[3 * g] = (uint8_t)(v >> 16);
        b[3 * g + 1] = (uint8_t)(v >> 8);
        if (g < 6)
            b[3 * g + 2] = (uint8_t)v;
    }
    auto be32 = [&](int o) {
        return ((uint32_t)b[o] << 24) | ((uint32_t)b[o + 1] << 16) | ((uint32_t)b[o + 2] << 8) | b[o + 3];
    };
    sid_out[i] = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    ts_out[i] = (int32_t)be32(4);
    int64_t sz = (int64_t)(((uint64_t)be32(8) << 32) | be32(12));
    // fdfs_get_file_info_ex (client/storage_client.c:2175-2214): an appender
    // (IS_APPENDER_FILE, INFINITE_FILE_SIZE = 2^58) is tested first and
    // reports size -1 and crc 0 (the memset FDFSFileInfo); a master file
    // keeps the low 32 bits when bit 63 (COMBINE_RAND_FILE_SIZE) or the trunk
    // mark (2^59, tracker/tracker_types.h:103) is set.
    uint32_t crc = be32(16);
    if (sz & (1ll << 58)) {
        sz = -1;
        crc = 0;
    } else if (((uint64_t)sz >> 63) || (sz & (1ll << 59))) {
        sz &= 0xFFFFFFFFll;
    }
    size_out[i] = sz;
    crc_out[i] = crc;
}

__device__ __forceinline__ void put_be32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

__global__ void trunk_pack_kernel(const uint8_t *__restrict__ type, const int32_t *__restrict__ alloc,
                                  const int32_t *__restrict__ size, const uint32_t *__restrict__ crc,
                                  const int32_t *__restrict__ mtime, const uint8_t *__restrict__ ext,
                                  uint32_t n, uint8_t *__restrict__ hdr)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    uint8_t h[24];
    h[0] = type[i];
    put_be32(h + 1, (uint32_t)alloc[i]);
    put_be32(h + 5, (uint32_t)size[i]);
    put_be32(h + 9, crc[i]);
    put_be32(h + 13, (uint32_t)mtime[i]);
#pragma unroll
    for (int k = 0; k < 7; k++)
        h[17 + k] = ext[7ull * i + k];
    uint8_t *o = hdr + 24ull * i;
#pragma unroll
    for (int k = 0; k < 24; k++)
        o[k] = h[k];
}

__global__ void trunk_unpack_kernel(const uint8_t *__restrict__ hdr, uint32_t n,
                                    uint8_t *__restrict__ type, int32_t *__restrict__ alloc,
                                    int32_t *__restrict__ size, uint32_t *__restrict__ crc,
                                    int32_t *__restrict__ mtime, uint8_t *__restrict__ ext)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint8_t *h = hdr + 24ull * i;
    auto be32 = [&](int o) {
        return ((uint32_t)h[o] << 24) | ((uint32_t)h[o + 1] << 16) | ((uint32_t)h[o + 2] << 8) | h[o + 3];
    };
    type[i] = h[0];
    alloc[i] = (int32_t)be32(1);
    size[i] = (int32_t)be32(5);
    crc[i] = be32(9);
    mtime[i] = (int32_t)be32(13);
#pragma unroll
    for (int k = 0; k < 7; k++)
        ext[7ull * i + k] = h[17 + k];
}

// key = ns || 0x01 || obj_id; the namespace prefix's PJW state is computed
// once on the host (it is the same for every key) and passed as h0.  The
// obj ids are records of `stride` bytes (4-aligned), `lens[i]` (or `stride`)
// of them hashed: 24-byte signatures for the "fid" keys, file-id strings
// ("group/M00/..") for the "ref" and "sig" keys.
// dcount (device, optional): only the first *dcount records are live (the
// class sources of a recovery batch, counted on the device).
template <bool SAR>
__global__ void fdht_route_kernel(const uint8_t *__restrict__ keys, uint32_t stride,
                                  const uint32_t *__restrict__ lens, uint64_t n,
                                  const uint64_t *__restrict__ dcount, uint32_t h0,
                                  uint32_t group_count, const uint32_t *__restrict__ servers,
                                  int32_t *__restrict__ hash_out, uint32_t *__restrict__ group_out,
                                  uint32_t *__restrict__ server_out, uint32_t *__restrict__ gcount)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || (dcount && i >= *dcount))
        return;
    const uint32_t *p = reinterpret_cast<const uint32_t *>(keys + (uint64_t)stride * i);
    uint32_t len = lens ? lens[i] : stride;
    if (len > stride)
        len = stride;
    uint32_t h = pjw_step<SAR>(h0, 0x01u);  // FDHT_FULL_KEY_SEPERATOR
    uint32_t k = 0;
    for (; k + 4 <= len; k += 4) {
        const uint32_t v = p[k >> 2];
#pragma unroll
        for (int q = 0; q < 4; q++)
            h = pjw_step<SAR>(h, (v >> (8 * q)) & 0xFFu);
    }
    if (k < len) {
        const uint32_t v = p[k >> 2];
        for (int q = 0; k + q < len; q++)
            h = pjw_step<SAR>(h, (v >> (8 * q)) & 0xFFu);
    }
    const int32_t kh = (int32_t)h & 0x7FFFFFFF;  // CALC_KEY_HASH_CODE: clear the sign
    const uint32_t g = (uint32_t)kh % group_count;
    int32_t nh = (int32_t)(((uint32_t)kh << 16) | ((uint32_t)kh >> 16));
    if (nh < 0)
        nh &= 0x7FFFFFFF;
    const uint32_t cnt = servers ? servers[g] : 1u;
    hash_out[i] = kh;
    group_out[i] = g;
    server_out[i] = (uint32_t)nh % (cnt ? cnt : 1u);
    atomicAdd(&gcount[g], 1u);
}

__global__ void group_scan_kernel(const uint32_t *__restrict__ gcount, uint32_t group_count,
                                  uint64_t *__restrict__ start, uint64_t *__restrict__ cursor)
{
    // group_count is small (FastDHT groups): one thread scans
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        uint64_t run = 0;
        for (uint32_t g = 0; g < group_count; g++) {
            start[g] = run;
            cursor[g] = run;
            run += gcount[g];
        }
        start[group_count] = run;
    }
}

__global__ void group_scatter_kernel(const uint32_t *__restrict__ group, uint64_t n,
                                     const uint64_t *__restrict__ dcount,
                                     uint64_t *__restrict__ cursor, uint64_t *__restrict__ order)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || (dcount && i >= *dcount))
        return;
    const uint64_t pos = atomicAdd(reinterpret_cast<unsigned long long *>(&cursor[group[i]]), 1ull);
    order[pos] = i;
}

__global__ void scrub_kernel(const uint32_t *__restrict__ crc, const uint32_t *__restrict__ expect,
                             uint32_t n, uint8_t *__restrict__ bad, uint32_t *__restrict__ nbad)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const bool b = crc[i] != expect[i];
    bad[i] = b ? 1 : 0;
    if (b)
        atomicAdd(nbad, 1u);
}

// ------------------------------------------------------------------ launchers

static inline unsigned blocks(uint64_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

hipError_t launch_file_ids(bool sar, uint32_t server_id, const uint32_t *crc32, const int64_t *size,
                           const int32_t *ts, const uint32_t *rnd, uint32_t n, uint32_t subdirs,
                           char *name_out, uint8_t *sub_out, hipStream_t st)
{
    if (sar)
        file_id_kernel<true><<<blocks(n, 256), 256, 0, st>>>(server_id, crc32, size, ts, rnd, n,
                                                            subdirs, name_out, sub_out);
    else
        file_id_kernel<false><<<blocks(n, 256), 256, 0, st>>>(server_id, crc32, size, ts, rnd, n,
                                                             subdirs, name_out, sub_out);
    return hipGetLastError();
}

hipError_t launch_parse_file_ids(const uint8_t *names, uint32_t n, uint32_t *sid, int32_t *ts,
                                 int64_t *size, uint32_t *crc, hipStream_t st)
{
    parse_file_id_kernel<<<blocks(n, 256), 256, 0, st>>>(names, n, sid, ts, size, crc);
    return hipGetLastError();
}

hipError_t launch_trunk_pack(const uint8_t *type, const int32_t *alloc, const int32_t *size,
                             const uint32_t *crc, const int32_t *mtime, const uint8_t *ext,
                             uint32_t n, uint8_t *hdr, hipStream_t st)
{
    trunk_pack_kernel<<<blocks(n, 256), 256, 0, st>>>(type, alloc, size, crc, mtime, ext, n, hdr);
    return hipGetLastError();
}

hipError_t launch_trunk_unpack(const uint8_t *hdr, uint32_t n, uint8_t *type, int32_t *alloc,
                               int32_t *size, uint32_t *crc, int32_t *mtime, uint8_t *ext,
                               hipStream_t st)
{
    trunk_unpack_kernel<<<blocks(n, 256), 256, 0, st>>>(hdr, n, type, alloc, size, crc, mtime, ext);
    return hipGetLastError();
}

uint32_t pjw_prefix(bool sar, const char *ns, int len)
{
    uint32_t h = 0;
    for (int k = 0; k < len; k++) {
        h = (h << 4) + (uint8_t)ns[k];
        const uint32_t x = h & 0xF0000000u;
        if (x)
            h = (h ^ (sar ? (uint32_t)((int32_t)x >> 24) : (x >> 24))) & 0x0FFFFFFFu;
    }
    return h;
}

hipError_t launch_fdht_route(bool sar, const uint8_t *keys, uint32_t stride, const uint32_t *lens,
                             uint64_t n, const uint64_t *dcount, uint32_t h0, uint32_t group_count,
                             const uint32_t *servers, int32_t *hash_out, uint32_t *group_out,
                             uint32_t *server_out, uint32_t *gcount, uint64_t *start,
                             uint64_t *cursor, uint64_t *order, hipStream_t st)
{
    hipError_t e = launch_zero_u32(gcount, group_count, st);
    if (e != hipSuccess)
        return e;
    if (n && sar)
        fdht_route_kernel<true><<<blocks(n, 256), 256, 0, st>>>(keys, stride, lens, n, dcount, h0,
                                                               group_count, servers, hash_out, group_out,
                                                               server_out, gcount);
    else if (n)
        fdht_route_kernel<false><<<blocks(n, 256), 256, 0, st>>>(keys, stride, lens, n, dcount, h0,
                                                                group_count, servers, hash_out,
                                                                group_out, server_out, gcount);
    group_scan_kernel<<<1, 64, 0, st>>>(gcount, group_count, start, cursor);
    if (order && n)
        group_scatter_kernel<<<blocks(n, 256), 256, 0, st>>>(group_out, n, dcount, cursor, order);
    return hipGetLastError();
}

// ---- recovery batch: the class sources, compacted on the device ----------

__global__ void source_flag_kernel(const uint64_t *__restrict__ rep, uint64_t n,
                                   uint64_t *__restrict__ flag, uint64_t *__restrict__ iota)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    flag[i] = rep[i] == i ? 1u : 0u;  // the first file of its class (A9 "fid" source)
    iota[i] = i;
}

// pos: exclusive scan of flag (pos[n] = number of sources)
__global__ void source_compact_kernel(const uint64_t *__restrict__ flag, const uint64_t *__restrict__ pos,
                                      uint64_t n, const uint8_t *__restrict__ sig,
                                      const uint8_t *__restrict__ ids, uint32_t stride,
                                      const uint32_t *__restrict__ lens, uint64_t *__restrict__ index,
                                      uint8_t *__restrict__ csig, uint8_t *__restrict__ cids,
                                      uint32_t *__restrict__ clens, uint64_t *__restrict__ nsrc)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0)
        *nsrc = pos[n];
    if (i >= n || !flag[i])
        return;
    const uint64_t k = pos[i];
    index[k] = i;
    const uint2 *s = reinterpret_cast<const uint2 *>(sig + 24 * i);
    uint2 *d = reinterpret_cast<uint2 *>(csig + 24 * k);
    d[0] = s[0];
    d[1] = s[1];
    d[2] = s[2];
    const uint32_t *a = reinterpret_cast<const uint32_t *>(ids + (uint64_t)stride * i);
    uint32_t *b = reinterpret_cast<uint32_t *>(cids + (uint64_t)stride * k);
    for (uint32_t w = 0; w < stride / 4; w++)
        b[w] = a[w];
    clens[k] = lens ? lens[i] : stride;
}

hipError_t launch_sources(const uint64_t *rep, uint64_t n, const uint8_t *sig, const uint8_t *ids,
                          uint32_t stride, const uint32_t *lens, uint64_t *flag, uint64_t *pos,
                          uint64_t *bsum, uint64_t *iota, uint64_t *index, uint8_t *csig,
                          uint8_t *cids, uint32_t *clens, uint64_t *nsrc, hipStream_t st)
{
    source_flag_kernel<<<blocks(n, 256), 256, 0, st>>>(rep, n, flag, iota);
    hipError_t e = launch_exclusive_scan(flag, n, pos, bsum, st);
    if (e != hipSuccess)
        return e;
    source_compact_kernel<<<blocks(n, 256), 256, 0, st>>>(flag, pos, n, sig, ids, stride, lens, index,
                                                          csig, cids, clens, nsrc);
    return hipGetLastError();
}

hipError_t launch_scrub(const uint32_t *crc, const uint32_t *expect, uint32_t n, uint8_t *bad,
                        uint32_t *nbad, hipStream_t st)
{
    hipError_t e = launch_zero_u32(nbad, 1, st);
    if (e != hipSuccess)
        return e;
    scrub_kernel<<<blocks(n, 256), 256, 0, st>>>(crc, expect, n, bad, nbad);
    return hipGetLastError();
}

}  // namespace fdfs
