// libfdfs_gpu bulk duplicate grouping (gfx950).
//
// Replaces the per-file FastDHT round trips of the upload-done handler
// (storage/storage_service.c:2652 get "fid", :2714 set "fid", :2734 set "ref",
// :2984 inc "ref") for bulk / recovery ingest.  Output per record, in input
// order: rep = smallest ingest index with the same 24-byte signature (the
// file that became the "fid" source), ref = number of records sharing it
// (the "ref" count after every link).
//
//  * dedup_bucket: owner rank = hash(sig) mod nranks; rows {sig[24], gidx}
//    packed per owner for one all-to-all over RCCL (the FastDHT key
//    partition, storage/fdht_client/fdht_client.c:301-305, re-expressed as a
//    GPU bucket).
//  * dedup_group: on the owner, a lock-free open-addressing table keyed by the
//    full 24 bytes: a slot is claimed by CAS of a record index and never
//    changes, so a probe compares the immutable signature bytes of the
//    claiming record; class min(gidx) and size via 64/32-bit atomics.
#include "fdfs_device.hpp"
#include "fdfs_kernels.hpp"

namespace fdfs {

constexpr uint32_t kEmpty = 0xFFFFFFFFu;

__device__ __forceinline__ uint64_t fmix64(uint64_t k)
{
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

__device__ __forceinline__ void load_sig(const uint8_t *row, uint64_t &a, uint64_t &b, uint64_t &c)
{
    const uint64_t *p = reinterpret_cast<const uint64_t *>(row);
    a = p[0];
    b = p[1];
    c = p[2];
}

__device__ __forceinline__ uint64_t sig_hash(uint64_t a, uint64_t b, uint64_t c)
{
    return fmix64(a ^ fmix64(b ^ fmix64(c + 0x9E3779B97F4A7C15ull)));
}

__global__ void dedup_insert_kernel(const uint8_t *__restrict__ sig, uint32_t sig_stride,
                                    const uint64_t *__restrict__ gidx, uint32_t gidx_stride,
                                    uint64_t n, uint32_t *__restrict__ slots,
                                    uint64_t *__restrict__ minidx, uint32_t *__restrict__ count,
                                    uint32_t *__restrict__ slot_of, uint64_t mask)
{
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t a, b, c;
        load_sig(sig + r * sig_stride, a, b, c);
        uint64_t pos = sig_hash(a, b, c) & mask;
        for (;;) {
            uint32_t cur = __hip_atomic_load(&slots[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == kEmpty) {
                cur = atomicCAS(&slots[pos], kEmpty, (uint32_t)r);
                if (cur == kEmpty)
                    break;  // claimed
            }
            uint64_t a2, b2, c2;
            load_sig(sig + (uint64_t)cur * sig_stride, a2, b2, c2);
            if (a2 == a && b2 == b && c2 == c)
                break;  // same signature class
            pos = (pos + 1) & mask;
        }
        const uint64_t g = gidx_stride ? gidx[r * gidx_stride] : r;
        atomicMin(reinterpret_cast<unsigned long long *>(&minidx[pos]), (unsigned long long)g);
        atomicAdd(&count[pos], 1u);
        slot_of[r] = (uint32_t)pos;
    }
}

__global__ void dedup_emit_kernel(uint64_t n, const uint32_t *__restrict__ slot_of,
                                  const uint64_t *__restrict__ minidx,
                                  const uint32_t *__restrict__ count, uint64_t *__restrict__ rep_out,
                                  uint32_t *__restrict__ ref_out)
{
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = slot_of[r];
        rep_out[r] = minidx[s];
        ref_out[r] = count[s];
    }
}

uint64_t dedup_table_slots(uint64_t n)
{
    uint64_t c = 1024;
    while (c < 2 * n)
        c <<= 1;
    return c;
}

static unsigned grid_for(uint64_t n, unsigned block)
{
    uint64_t g = (n + block - 1) / block;
    if (g > 16384)
        g = 16384;
    return g ? (unsigned)g : 1u;
}

hipError_t launch_dedup_group(const uint8_t *sig, uint32_t sig_stride, const uint64_t *gidx,
                              uint32_t gidx_stride, uint64_t n, uint32_t *slots, uint64_t *minidx,
                              uint32_t *count, uint32_t *slot_of, uint64_t nslots,
                              uint64_t *rep_out, uint32_t *ref_out, hipStream_t st, hipEvent_t ev0,
                              hipEvent_t ev1)
{
    if (n == 0)
        return hipSuccess;
    hipError_t e;
    if ((e = hipMemsetAsync(slots, 0xFF, nslots * sizeof(uint32_t), st)) != hipSuccess)
        return e;
    if ((e = hipMemsetAsync(minidx, 0xFF, nslots * sizeof(uint64_t), st)) != hipSuccess)
        return e;
    if ((e = hipMemsetAsync(count, 0, nslots * sizeof(uint32_t), st)) != hipSuccess)
        return e;
    if (ev0)
        (void)hipEventRecord(ev0, st);
    dedup_insert_kernel<<<grid_for(n, 256), 256, 0, st>>>(sig, sig_stride, gidx, gidx_stride, n,
                                                          slots, minidx, count, slot_of, nslots - 1);
    dedup_emit_kernel<<<grid_for(n, 256), 256, 0, st>>>(n, slot_of, minidx, count, rep_out, ref_out);
    if (ev1)
        (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

// ------------------------------------------------------------------ bucket

__device__ __forceinline__ uint32_t owner_of(const uint8_t *row, uint32_t nranks)
{
    uint64_t a, b, c;
    load_sig(row, a, b, c);
    return (uint32_t)((sig_hash(a, b, c) >> 32) % nranks);
}

__global__ void bucket_count_kernel(const uint8_t *__restrict__ sig, uint64_t n, uint32_t nranks,
                                    uint64_t *__restrict__ counts)
{
    __shared__ uint32_t h[64];
    for (int k = threadIdx.x; k < 64; k += blockDim.x)
        h[k] = 0;
    __syncthreads();
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (uint64_t)gridDim.x * blockDim.x)
        atomicAdd(&h[owner_of(sig + 24 * r, nranks)], 1u);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nranks; k += blockDim.x)
        if (h[k])
            atomicAdd(reinterpret_cast<unsigned long long *>(&counts[k]), (unsigned long long)h[k]);
}

__global__ void bucket_scatter_kernel(const uint8_t *__restrict__ sig, const uint64_t *__restrict__ gidx,
                                      uint64_t n, uint32_t nranks, const uint64_t *__restrict__ counts,
                                      uint64_t *__restrict__ cursor, uint8_t *__restrict__ rows,
                                      uint64_t *__restrict__ row_of)
{
    __shared__ uint32_t cnt[64];
    __shared__ uint64_t bas[64];
    __shared__ uint64_t start[64];
    if (threadIdx.x == 0) {
        uint64_t run = 0;
        for (uint32_t k = 0; k < nranks; k++) {
            start[k] = run;
            run += counts[k];
        }
    }
    for (uint64_t r0 = (uint64_t)blockIdx.x * blockDim.x; r0 < n; r0 += (uint64_t)gridDim.x * blockDim.x) {
        for (int k = threadIdx.x; k < 64; k += blockDim.x)
            cnt[k] = 0;
        __syncthreads();
        const uint64_t r = r0 + threadIdx.x;
        uint32_t own = 0, rank = 0;
        if (r < n) {
            own = owner_of(sig + 24 * r, nranks);
            rank = atomicAdd(&cnt[own], 1u);
        }
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nranks; k += blockDim.x)
            if (cnt[k])
                bas[k] = start[k] + atomicAdd(reinterpret_cast<unsigned long long *>(&cursor[k]),
                                              (unsigned long long)cnt[k]);
        __syncthreads();
        if (r < n) {
            const uint64_t pos = bas[own] + rank;
            const uint64_t *s = reinterpret_cast<const uint64_t *>(sig + 24 * r);
            uint64_t *d = reinterpret_cast<uint64_t *>(rows + 32 * pos);
            d[0] = s[0];
            d[1] = s[1];
            d[2] = s[2];
            d[3] = gidx ? gidx[r] : r;
            if (row_of)
                row_of[r] = pos;
        }
        __syncthreads();
    }
}

hipError_t launch_dedup_bucket(const uint8_t *sig, const uint64_t *gidx, uint64_t n,
                               uint32_t nranks, uint8_t *records_out, uint64_t *counts_out,
                               uint64_t *cursor, uint64_t *row_of_out, hipStream_t st,
                               hipEvent_t ev0, hipEvent_t ev1)
{
    hipError_t e;
    if ((e = hipMemsetAsync(counts_out, 0, nranks * sizeof(uint64_t), st)) != hipSuccess)
        return e;
    if ((e = hipMemsetAsync(cursor, 0, nranks * sizeof(uint64_t), st)) != hipSuccess)
        return e;
    if (n == 0)
        return hipSuccess;
    if (ev0)
        (void)hipEventRecord(ev0, st);
    bucket_count_kernel<<<grid_for(n, 256), 256, 0, st>>>(sig, n, nranks, counts_out);
    bucket_scatter_kernel<<<grid_for(n, 256), 256, 0, st>>>(sig, gidx, n, nranks, counts_out, cursor,
                                                            records_out, row_of_out);
    if (ev1)
        (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

}  // namespace fdfs
