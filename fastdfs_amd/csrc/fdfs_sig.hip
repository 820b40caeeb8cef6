// libfdfs_gpu: segmented CRC32 kernel, planning kernels and launchers (gfx950).
//
//  * crc_seg_kernel<SAR>: CRC32 only (the default upload path and the
//    CRC of the MD5 method), one WAVE per kSegBytes segment of a file,
//    coalesced 4 KiB strides, conflict-free rotated slice-by-8 tables in LDS
//    (the byte-table slice-by-16 form measured slower), a 6-level GF(2) combine across
//    the wave, and a GF(2) matrix-power advance to combine segments of large
//    files.
//  * planning kernels: size-bin counting sort (lane-per-file paths), per-file
//    segment counts + exclusive scan (segment path).
//  * launch_sig_lane dispatches the lane-per-file paths: sig_hash_kernel
//    (fdfs_hash.hip, FDFS_SIG_HASH) and md5_stage_kernel (fdfs_md5.hip).
//
// Reference call sites replaced: storage/storage_dio.c:465-515 (CRC32_ex,
// CALC_HASH_CODES4, my_md5_update, *_FINAL) and
// storage/storage_service.c:106-120 (STORAGE_GEN_FILE_SIGNATURE).
#include "fdfs_device.hpp"
#include "fdfs_kernels.hpp"
#include "fdfs_segcrc.hpp"

namespace fdfs {

// ------------------------------------------------------- segmented CRC path
// (device helpers in fdfs_segcrc.hpp)

constexpr uint32_t kSegRingBytes = (kSegBlock / 64) * kFoldRingBytes;  // dynamic LDS: the waves' fold rings

template <bool SAR>
__global__ __launch_bounds__(kSegBlock) void crc_seg_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint64_t *__restrict__ sizes, const uint64_t *__restrict__ seg_first, uint32_t n_host,
    const uint32_t *__restrict__ n_dev, const DevTables *__restrict__ tabs, uint32_t *__restrict__ crc_out)
{
    const uint32_t n = n_dev ? *n_dev : n_host;  // file count, or written by big_plan_kernel
    const uint64_t total = seg_first[n];
    {  // a workgroup none of whose waves has a segment (small batches) skips the table fill
        const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6), w0 = (uint64_t)blockIdx.x * (blockDim.x >> 6);
        if ((total * w0) / nw == (total * (w0 + (blockDim.x >> 6))) / nw)
            return;
    }
    // the plain slice-by-16 tables (the signed variant's data is complemented
    // before the fold; only the runs' last vectors use them), the 4032-byte
    // advance and the byte table in LDS; the reduction tables stay in global
    // memory (24 lookups per run)
    __shared__ uint32_t smem[16 * 256 + 4 * 256 + 256];
    static_assert(sizeof(smem) + kSegRingBytes <= 160 * 1024, "one workgroup's LDS fits the CU's 160 KiB");
    uint32_t *sD = smem, *sA = smem + 16 * 256, *sT = sA + 4 * 256;
    const uint32_t *sR = &tabs->t.ADVRED[0][0][0];
    lds_fill(sD, &tabs->t.D[0][0], 16 * 256);
    lds_fill(sA, &tabs->t.ADV4032[0][0], 4 * 256);
    lds_fill(sT, tabs->t.T, 256);
    __syncthreads();

    const uint32_t K16 = tabs->t.K16;
    const int lane = threadIdx.x & 63;
    const uint64_t wpb = blockDim.x >> 6;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t w = (uint64_t)blockIdx.x * wpb + wv;
    const uint64_t nw = (uint64_t)gridDim.x * wpb;
    uint64_t s = (total * w) / nw;
    const uint64_t s_end = (total * (w + 1)) / nw;
    if (s >= s_end)
        return;
    // this wave's fold ring (kFoldRingBytes of the dynamic LDS)
    extern __shared__ __attribute__((aligned(16))) uint4 fold_ring[];
    uint4 *ring = fold_ring + (size_t)wv * kFoldSlots;
    const uint32_t ring_lds = lds_addr(ring);
    uint32_t lo = 0, hi = n;  // last f with seg_first[f] <= s
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (seg_first[mid] <= s)
            lo = mid;
        else
            hi = mid;
    }
    uint32_t f = lo;
    // The wave's segments are consecutive: each run of segments of one file
    // is one contiguous byte range, folded as one stream (crc_run); a run
    // that is the whole file stores its CRC, any other is advanced to the
    // file end (GF(2) matrix powers) and merged into crc_out by XOR.
    while (s < s_end) {
        while (seg_first[f + 1] <= s)
            f++;
        const uint64_t k0 = s - seg_first[f];
        const uint64_t s_stop = seg_first[f + 1] < s_end ? seg_first[f + 1] : s_end;
        const uint64_t L = sizes[f];
        const uint64_t lo_b = k0 * kSegBytes;
        const uint64_t hi_b = (L < (s_stop - seg_first[f]) * kSegBytes) ? L : (s_stop - seg_first[f]) * kSegBytes;
        const uint32_t v = crc_run<SAR>(sD, sA, sT, sR, K16, base + offs[f] + lo_b, hi_b - lo_b, k0 == 0, ring,
                                        ring_lds, lane);
        const uint32_t cl = k0 == 0 ? crc_final_const<SAR>(L) : 0u;
        if (k0 == 0 && hi_b == L) {
            if (lane == 0)
                crc_out[f] = v ^ cl;
        } else {
            const uint32_t u = advance_any(tabs, v, L - hi_b, lane);
            if (lane == 0)
                atomicXor(&crc_out[f], u ^ cl);
        }
        s = s_stop;
    }
}

// crc_tab_kernel<SAR>: the table fold, for files below kFoldMinBytes (the
// sparse fold's per-run costs -- its remainder, its ring's first steps --
// would dominate there).  One wave per kSegBytes segment range, each lane
// 64 B of every 4 KiB block with the rotated, replicated slice-by-8 tables,
// a 6-level GF(2) combine across the wave; a wave's consecutive segments of
// one file chain with the one-segment advance (ADVSEG).
template <bool SAR>
__global__ __launch_bounds__(kSegBlock) void crc_tab_kernel(
    const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
    const uint64_t *__restrict__ sizes, const uint64_t *__restrict__ seg_first, uint32_t n_host,
    const uint32_t *__restrict__ n_dev, const DevTables *__restrict__ tabs, uint32_t *__restrict__ crc_out)
{
    const uint32_t n = n_dev ? *n_dev : n_host;  // file count, or written by big_plan_kernel
    const uint64_t total = seg_first[n];
    {  // a workgroup none of whose waves has a segment (small batches) skips the table fill
        const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6), w0 = (uint64_t)blockIdx.x * (blockDim.x >> 6);
        if ((total * w0) / nw == (total * (w0 + (blockDim.x >> 6))) / nw)
            return;
    }
    // the 64 KiB conflict-free tables in LDS; the reduction tables stay in
    // global memory (24 lookups per segment)
    constexpr int kD = kRep8Dwords;
    __shared__ uint32_t smem[kD + 256 + 2 * 4 * 256];
    uint32_t *sD = smem, *sT = smem + kD, *sA = sT + 256, *sS = sA + 1024;
    const uint32_t *sR = &tabs->t.ADVRED[0][0][0];
    lds_fill(sS, &tabs->t.ADVSEG[0][0], 4 * 256);
    lds_fill_rep8(sD, SAR ? &tabs->Dc[0][0] : &tabs->t.D[0][0]);
    lds_fill(sT, tabs->t.T, 256);
    lds_fill(sA, &tabs->t.ADV4032[0][0], 4 * 256);
    __syncthreads();

    const uint32_t K8 = tabs->t.K8;
    const Rep8Lane R8 = rep8_lane(threadIdx.x & 63);
    const int lane = threadIdx.x & 63;
    const uint64_t wpb = blockDim.x >> 6;
    const uint64_t w = (uint64_t)blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * wpb;
    uint64_t s = (total * w) / nw;
    const uint64_t s_end = (total * (w + 1)) / nw;
    if (s >= s_end)
        return;
    uint32_t lo = 0, hi = n;  // last f with seg_first[f] <= s
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (seg_first[mid] <= s)
            lo = mid;
        else
            hi = mid;
    }
    uint32_t f = lo;
    // The wave's segments are consecutive, so a run of segments of one file
    // is chained in place (state = ADV_seg(state) ^ crc0(seg), one 4-lookup
    // advance per segment); only when the run ends is the state advanced to
    // the file end (GF(2) matrix powers) and merged into crc_out.
    uint32_t run_f = 0xFFFFFFFFu, run_state = 0;
    uint64_t run_end = 0;
    bool run_has_first = false, run_whole = false;
    for (;; s++) {
        const bool more = s < s_end;
        if (more) {
            while (seg_first[f + 1] <= s)
                f++;
        }
        if (run_f != 0xFFFFFFFFu && (!more || f != run_f)) {  // flush the finished run
            const uint64_t L = sizes[run_f];
            const uint32_t cl = run_has_first ? crc_final_const<SAR>(L) : 0u;
            if (run_whole) {
                if (lane == 0)
                    crc_out[run_f] = run_state ^ cl;
            } else {
                const uint32_t v = advance_any(tabs, run_state, L - run_end, lane);
                if (lane == 0)
                    atomicXor(&crc_out[run_f], v ^ cl);
            }
            run_f = 0xFFFFFFFFu;
        }
        if (!more)
            break;
        const uint64_t k = s - seg_first[f];
        const uint64_t nseg = seg_first[f + 1] - seg_first[f];
        const uint64_t L = sizes[f];
        const uint8_t *fp = base + offs[f];
        const uint64_t lo_b = k * kSegBytes;
        const uint64_t hi_b = (L < lo_b + kSegBytes) ? L : lo_b + kSegBytes;
        const uint32_t v = crc_segment<SAR>(sD, sT, sA, sR, R8, K8, fp + lo_b, hi_b - lo_b, k == 0, lane);
        if (run_f == f) {
            const uint64_t len = hi_b - lo_b;
            const uint32_t adv = (len == kSegBytes) ? apply4(sS, run_state)
                                                    : advance_any(tabs, run_state, len, lane);
            run_state = adv ^ v;
        } else {
            run_f = f;
            run_state = v;
            run_has_first = (k == 0);
        }
        run_end = hi_b;
        run_whole = run_has_first && (k + 1 == nseg);
    }
}

// ---------------------------------------------------------------- planning

// Batches of at most kPlanSmall files: segment counts, their exclusive scans
// (seg_first[0..n] of the table kernel's list, seg_first[n + 1 ..] of the
// fold kernel's: a file's segments are in one of them) and the zeroed CRC
// slots in one workgroup, instead of plan_nseg_kernel + two three-kernel
// scans (a small call is launch-bound).
constexpr int kPlanSmallItems = 4;
constexpr uint32_t kPlanSmall = 1024 * kPlanSmallItems;

__device__ __forceinline__ uint64_t block_scan_u64(uint64_t x, uint64_t *wsum)  // exclusive, 1024 threads
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t mine = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= o)
            x += y;
    }
    if (lane == 63)
        wsum[wid] = x;
    __syncthreads();
    uint64_t run = x - mine;
    for (int k = 0; k < wid; k++)
        run += wsum[k];
    __syncthreads();
    return run;
}

__global__ __launch_bounds__(1024) void plan_small_kernel(const uint64_t *__restrict__ sizes, uint32_t n,
                                                          uint64_t *__restrict__ seg_first,
                                                          uint32_t *__restrict__ crc_out)
{
    __shared__ uint64_t wsum[16];
    const uint32_t i0 = threadIdx.x * kPlanSmallItems;
    uint64_t vt[kPlanSmallItems], vf[kPlanSmallItems], xt = 0, xf = 0;
#pragma unroll
    for (int k = 0; k < kPlanSmallItems; k++) {
        const uint64_t L = i0 + k < n ? sizes[i0 + k] : 0;
        const uint64_t c = (L + kSegBytes - 1) / kSegBytes;
        vt[k] = L < kFoldMinBytes ? c : 0;
        vf[k] = L < kFoldMinBytes ? 0 : c;
        xt += vt[k];
        xf += vf[k];
        if (i0 + k < n)
            crc_out[i0 + k] = 0;  // empty files keep CRC 0; multi-segment files accumulate by XOR
    }
    uint64_t rt = block_scan_u64(xt, wsum), rf = block_scan_u64(xf, wsum);
#pragma unroll
    for (int k = 0; k < kPlanSmallItems; k++) {
        if (i0 + k <= n) {
            seg_first[i0 + k] = rt;  // seg_first[n] = the total
            seg_first[n + 1 + i0 + k] = rf;
        }
        rt += vt[k];
        rf += vf[k];
    }
}

__global__ void plan_nseg_kernel(const uint64_t *__restrict__ sizes, uint32_t n,
                                 uint64_t *__restrict__ nseg, uint32_t *__restrict__ crc_out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t L = sizes[i];
    const uint64_t c = (L + kSegBytes - 1) / kSegBytes;
    nseg[i] = L < kFoldMinBytes ? c : 0;  // the table kernel's list
    nseg[n + i] = L < kFoldMinBytes ? 0 : c;  // the fold kernel's
    crc_out[i] = 0;  // empty files keep CRC 0; multi-segment files accumulate by XOR
}

__device__ __forceinline__ uint32_t size_bin(uint64_t L)
{
    if (L == 0)
        return 0;
    const uint32_t e = 63 - __builtin_clzll(L);
    const uint32_t m = (e >= 5) ? (uint32_t)((L >> (e - 5)) & 31u) : (uint32_t)((L << (5 - e)) & 31u);
    return e * 32 + m;  // < kSizeBins
}

__global__ void bin_hist_kernel(const uint64_t *__restrict__ sizes, uint32_t n,
                                uint32_t *__restrict__ hist, uint32_t bmask)
{
    __shared__ uint32_t h[kSizeBins];
    for (int b = threadIdx.x; b < kSizeBins; b += blockDim.x)
        h[b] = 0;
    __syncthreads();
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        atomicAdd(&h[size_bin(sizes[i]) & bmask], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < kSizeBins; b += blockDim.x)
        if (h[b])
            atomicAdd(&hist[b], h[b]);
}

// Descending exclusive scan of the bin histogram (one block of kSizeBins / 2
// threads, two bins each: wave shuffles, then the waves' totals).
__global__ __launch_bounds__(1024) void bin_scan_kernel(const uint32_t *__restrict__ hist,
                                                        uint32_t *__restrict__ cursor)
{
    static_assert(kSizeBins == 2 * 1024, "two bins per thread");
    __shared__ uint32_t wsum[16];
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    // thread t owns reversed positions 2t, 2t + 1 (largest bin first)
    const uint32_t a = hist[kSizeBins - 1 - 2 * t], b = hist[kSizeBins - 2 - 2 * t];
    uint32_t x = a + b;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o)
            x += y;
    }
    if (lane == 63)
        wsum[wid] = x;
    __syncthreads();
    uint32_t run = x - (a + b);
    for (int k = 0; k < wid; k++)
        run += wsum[k];
    cursor[kSizeBins - 1 - 2 * t] = run;
    cursor[kSizeBins - 2 - 2 * t] = run + a;
}

// kBinItems files per thread: each block reserves its bins' ranges with one
// global atomic per non-empty bin, so fewer, fuller blocks mean fewer atomics
// on the same ~100 hot bins (one file per thread: ~1K blocks and 23 us per
// 1M files, most of it same-address atomics in L2).
constexpr int kBinItems = 8;

__global__ __launch_bounds__(1024) void bin_scatter_kernel(const uint64_t *__restrict__ sizes,
                                                           uint32_t n, uint32_t *__restrict__ cursor,
                                                           uint32_t *__restrict__ order, uint32_t *__restrict__ err,
                                                           uint32_t bmask)
{
    __shared__ uint32_t cnt[kSizeBins];
    __shared__ uint32_t bas[kSizeBins];
    for (int b = threadIdx.x; b < kSizeBins; b += blockDim.x)
        cnt[b] = 0;
    __syncthreads();
    const uint32_t i0 = blockIdx.x * (blockDim.x * kBinItems) + threadIdx.x;
    uint32_t bin[kBinItems], rank[kBinItems];
#pragma unroll
    for (int k = 0; k < kBinItems; k++) {
        const uint32_t i = i0 + k * blockDim.x;
        bin[k] = i < n ? (size_bin(sizes[i]) & bmask) : 0u;
    }
#pragma unroll
    for (int k = 0; k < kBinItems; k++)
        if (i0 + k * blockDim.x < n)
            rank[k] = atomicAdd(&cnt[bin[k]], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < kSizeBins; b += blockDim.x)
        if (cnt[b])
            bas[b] = atomicAdd(&cursor[b], cnt[b]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kBinItems; k++) {
        const uint32_t i = i0 + k * blockDim.x;
        if (i < n) {
            // a histogram that held counts before this batch's shifts the
            // cursors: a position past n is an error, never a store
            const uint32_t pos = bas[bin[k]] + rank[k];
            if (pos < n)
                order[pos] = i;
            else
                atomicOr(err, 1u);
        }
    }
}

// -------------------------------------------------------- exclusive scan u64

constexpr int kScanBlock = 256;
constexpr int kScanItems = 4;
constexpr int kScanTile = kScanBlock * kScanItems;

__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t *wsum, uint64_t &total)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= o)
            x += y;
    }
    if (lane == 63)
        wsum[wid] = x;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); k++) {
        if (k < wid)
            pre += wsum[k];
        tot += wsum[k];
    }
    __syncthreads();
    total = tot;
    return pre + x - v;
}

__global__ __launch_bounds__(kScanBlock) void scan_reduce_kernel(const uint64_t *__restrict__ in,
                                                                 uint64_t n,
                                                                 uint64_t *__restrict__ bsum)
{
    __shared__ uint64_t wsum[kScanBlock / 64];
    const uint64_t b0 = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint64_t vals[kScanItems], v = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; k++)  // branch-free loads, one wait
        vals[k] = in[b0 + k < n ? b0 + k : n - 1];
#pragma unroll
    for (int k = 0; k < kScanItems; k++)
        v += (b0 + k < n) ? vals[k] : 0;
    uint64_t tot;
    block_exclusive_scan(v, wsum, tot);
    if (threadIdx.x == 0)
        bsum[blockIdx.x] = tot;
}

// One block of 1024 threads, 4 sums per thread per pass (a 1.5K-sum scan is
// one pass: 11.3 us with 256 threads and one sum per thread per pass).
__global__ __launch_bounds__(1024) void scan_sums_kernel(uint64_t *__restrict__ bsum, uint64_t nb)
{
    constexpr int kI = 4;
    __shared__ uint64_t wsum[1024 / 64];
    uint64_t carry = 0;
    for (uint64_t c0 = 0; c0 < nb; c0 += 1024 * kI) {
        const uint64_t b0 = c0 + (uint64_t)threadIdx.x * kI;
        uint64_t vals[kI], v = 0;
#pragma unroll
        for (int k = 0; k < kI; k++)
            vals[k] = bsum[b0 + k < nb ? b0 + k : nb - 1];
#pragma unroll
        for (int k = 0; k < kI; k++) {
            vals[k] = (b0 + k < nb) ? vals[k] : 0;
            v += vals[k];
        }
        uint64_t tot;
        uint64_t run = carry + block_exclusive_scan(v, wsum, tot);
#pragma unroll
        for (int k = 0; k < kI; k++) {
            if (b0 + k < nb)
                bsum[b0 + k] = run;
            run += vals[k];
        }
        carry += tot;
    }
}

__global__ __launch_bounds__(kScanBlock) void scan_apply_kernel(const uint64_t *__restrict__ in,
                                                                uint64_t n,
                                                                const uint64_t *__restrict__ bsum,
                                                                uint64_t *__restrict__ out)
{
    __shared__ uint64_t wsum[kScanBlock / 64];
    const uint64_t b0 = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint64_t vals[kScanItems];
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; k++)  // branch-free loads, one wait
        vals[k] = in[b0 + k < n ? b0 + k : n - 1];
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        vals[k] = (b0 + k < n) ? vals[k] : 0;
        v += vals[k];
    }
    uint64_t tot;
    uint64_t run = bsum[blockIdx.x] + block_exclusive_scan(v, wsum, tot);
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        if (b0 + k < n)
            out[b0 + k] = run;
        run += vals[k];
    }
    if (b0 < n && b0 + kScanItems >= n)  // the thread holding the last element writes the total
        out[n] = run;
}

// ------------------------------------------------- big-file CRC offload (HASH)
// Files of >= T bytes (a power of two, so exactly the size bins from bin(T)
// up) are the first nbig entries of the size-descending order.  One block
// picks T, then lists them for crc_seg_kernel / poly_seg_kernel: compacted
// offsets/sizes, the exclusive scan of their segment counts, zeroed
// CRC and polynomial slots.
//
// Choosing T.  A batch of more than lat_files files puts several waves on a
// SIMD; the lane kernel is issue-bound there and T = kBigCrcMin for HASH
// (tuned on configs 1 and 2), no offload for MD5 (its fused CRC + MD5 pass
// is HBM-bound on config 3: a second pass would cost more than it saves).
// A smaller batch (the daemon's per-wakeup chunk batches,
// fdfs_gpu_update_batch) has at most one wave per SIMD, so the lane kernel
// lasts as long as its longest chain: kLanePs[method][0] per byte for a file
// hashed whole in its lane, kLanePs[method][1] for one whose CRC (and
// polynomials) are offloaded (measured: 256 KiB chunks alone,
// profiles/r02/chunk_sweep.txt; the 100 MiB file of config 1).  Offloading
// the files >= T adds their bytes to the segmented passes (kOffPs8 / 8 ps
// per byte: two passes for HASH, one for MD5).  T = 2^k (k in [kMinLog, 22])
// or no offload minimises max(chain below T, chain at or above T) + offload.
constexpr uint64_t kLanePs[2][2] = {{21000, 8600}, {20000, 11500}};  // [HASH, MD5][whole, offloaded]
constexpr uint64_t kOffPs8[2] = {4, 2};
constexpr int kMinLog = 13;

__device__ __forceinline__ uint64_t bin_hi(int b)  // an upper bound of the sizes in bin b
{
    if (b < 0)
        return 0;
    const int e = b >> 5, m = b & 31;
    if (e >= 35)
        return 1ull << 36;  // keeps the costs below far from overflow
    return e >= 5 ? (uint64_t)(33 + m) << (e - 5) : 1ull << (e + 1);
}
__device__ __forceinline__ uint64_t bin_lo(int b)
{
    const int e = b >> 5, m = b & 31;
    return e >= 5 ? (uint64_t)(32 + m) << (e - 5) : (uint64_t)b;
}

__global__ __launch_bounds__(1024) void big_plan_kernel(
    const uint32_t *__restrict__ hist, const uint32_t *__restrict__ order,
    const uint64_t *__restrict__ offs, const uint64_t *__restrict__ sizes, uint32_t n, int method,
    uint32_t lat_files, uint32_t *__restrict__ nbig_out, uint64_t *__restrict__ big_min,
    uint64_t *__restrict__ boffs, uint64_t *__restrict__ bsizes,
    uint64_t *__restrict__ seg_first, uint32_t *__restrict__ bcrc, uint32_t *__restrict__ bpoly,
    uint32_t *__restrict__ err)
{
    static_assert(kSizeBins == 2 * 1024, "two bins per thread");
    __shared__ uint32_t wsum[16];
    __shared__ uint64_t wsum64[16];
    __shared__ uint64_t eb[64];  // per exponent: bytes (from bin lower bounds)
    __shared__ int em[64];       // per exponent: largest nonempty bin, -1 if none
    __shared__ uint32_t nb_s, b0_s;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int mi = method == 2 ? 1 : 0;
    if (n > lat_files) {
        if (threadIdx.x == 0)
            b0_s = mi ? (uint32_t)kSizeBins  // MD5: no offload
                      : size_bin(method == 0 ? kFoldMinBytes : kBigCrcMin);  // CRC only: the fold's files
    } else {
        // thread t: bins 2t, 2t + 1, both of exponent t >> 4
        const int t = threadIdx.x;
        uint64_t by = 0;
        int mb = -1;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int b = 2 * t + k;
            const uint32_t c = hist[b];
            if (c) {
                by += (uint64_t)c * bin_lo(b);
                mb = b;
            }
        }
#pragma unroll
        for (int o = 8; o; o >>= 1) {
            by += __shfl_xor(by, o);
            const int y = __shfl_xor(mb, o);
            mb = y > mb ? y : mb;
        }
        if ((t & 15) == 0) {
            eb[t >> 4] = by;
            em[t >> 4] = mb;
        }
        __syncthreads();
        if (wid == 0) {  // lane = exponent k: the candidate T = 2^k
            const int k = lane;
            uint64_t above = eb[k];  // bytes in exponents >= k (suffix sum)
            int below = em[k];       // largest bin in exponents < k (exclusive prefix max)
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint64_t a = __shfl_down(above, o);
                if (lane + o < 64)
                    above += a;
            }
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(below, o);
                if (lane >= o)
                    below = y > below ? y : below;
            }
            below = __shfl_up(below, 1);
            if (lane == 0)
                below = -1;
            above = above < (1ull << 40) ? above : (1ull << 40);
            int top = em[k];
#pragma unroll
            for (int o = 32; o; o >>= 1) {
                const int y = __shfl_xor(top, o);
                top = y > top ? y : top;
            }
            // key = cost * 64 + (63 - k): the smallest cost, ties to the larger T
            const uint64_t whole = kLanePs[mi][0] * 8, lean = kLanePs[mi][1] * 8;  // 1/8 ps per byte
            const uint64_t none = bin_hi(top) * whole;
            uint64_t key = none * 64;  // k = 63: no offload
            if (k >= kMinLog && k <= 22) {
                const uint64_t chain_small = bin_hi(below) * whole;
                const uint64_t chain_big = (top >> 5) >= k ? bin_hi(top) * lean : 0;
                const uint64_t cost = (chain_small > chain_big ? chain_small : chain_big) + above * kOffPs8[mi];
                key = cost * 64 + (uint64_t)(63 - k);
            }
#pragma unroll
            for (int o = 32; o; o >>= 1) {
                const uint64_t y = __shfl_xor(key, o);
                key = y < key ? y : key;
            }
            if (lane == 0) {
                const int kb = 63 - (int)(key & 63);
                b0_s = kb >= 63 ? (uint32_t)kSizeBins : (uint32_t)(kb * 32);  // bin(2^kb)
            }
        }
    }
    __syncthreads();
    const uint32_t b0 = b0_s;
    if (threadIdx.x == 0)
        *big_min = b0 >= (uint32_t)kSizeBins ? ~0ull : bin_lo((int)b0);  // sizes in bins >= b0
    uint32_t cnt = 0;
    for (uint32_t b = b0 + threadIdx.x; b < kSizeBins; b += blockDim.x)
        cnt += hist[b];
#pragma unroll
    for (int o = 32; o; o >>= 1)
        cnt += __shfl_xor(cnt, o);
    if (lane == 0)
        wsum[wid] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int k = 0; k < (int)(blockDim.x >> 6); k++)
            t += wsum[k];
        nb_s = t < n ? t : n;
        *nbig_out = nb_s;
    }
    __syncthreads();
    const uint32_t nbig = nb_s;
    uint64_t carry = 0;
    for (uint32_t i0 = 0; i0 < nbig; i0 += blockDim.x) {
        const uint32_t i = i0 + threadIdx.x;
        uint64_t ns = 0;
        if (i < nbig) {
            const uint32_t f = order[i];
            const bool ok = f < n;  // a stale order entry: skipped (an empty file) and flagged
            if (!ok)
                atomicOr(err, 1u);
            const uint64_t L = ok ? sizes[f] : 0;
            boffs[i] = ok ? offs[f] : 0;
            bsizes[i] = L;
            bcrc[i] = 0;  // crc_seg_kernel accumulates multi-segment files by XOR
            bpoly[2ull * i] = 0;  // poly_seg_kernel adds segment contributions
            bpoly[2ull * i + 1] = 0;
            ns = (L + kSegBytes - 1) / kSegBytes;
        }
        uint64_t x = ns;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(x, o);
            if (lane >= o)
                x += y;
        }
        if (lane == 63)
            wsum64[wid] = x;
        __syncthreads();
        uint64_t before = carry;
        for (int k = 0; k < wid; k++)
            before += wsum64[k];
        if (i < nbig)
            seg_first[i] = before + x - ns;
        uint64_t tot = 0;
        for (int k = 0; k < (int)(blockDim.x >> 6); k++)
            tot += wsum64[k];
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0)
        seg_first[nbig] = carry;
}


// After the lane kernel: the big files' segmented CRC, simple_hash and
// Time33 into crc_out, their signature fields and codes[0], [2], [3].
__global__ void big_patch_kernel(const uint32_t *__restrict__ nbig, const uint32_t *__restrict__ order,
                                 uint32_t n, const uint32_t *__restrict__ bcrc, const uint32_t *__restrict__ bpoly,
                                 bool md5, uint32_t *__restrict__ crc_out, uint8_t *__restrict__ sig_out,
                                 int32_t *__restrict__ codes_out)
{
    const uint32_t nb = *nbig;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += gridDim.x * blockDim.x) {
        const uint32_t f = order[i], c = bcrc[i], s = bpoly[2ull * i], t = bpoly[2ull * i + 1];
        if (f >= n)  // flagged by big_plan_kernel
            continue;
        crc_out[f] = c;
        if (md5)  // the signature and codes hold the MD5 digest
            continue;
        if (sig_out) {  // be32 crc at 8, be32 simple at 16, be32 Time33 at 20
            uint32_t *sp = reinterpret_cast<uint32_t *>(sig_out + 24ull * f);
            sp[2] = bswap32(c);
            sp[4] = bswap32(s);
            sp[5] = bswap32(t);
        }
        if (codes_out) {
            codes_out[4ull * f] = (int32_t)c;
            codes_out[4ull * f + 2] = (int32_t)s;
            codes_out[4ull * f + 3] = (int32_t)t;
        }
    }
}

// The same for the chunked update (fdfs_gpu_update_batch): the segmented
// kernels hashed each big chunk from the one-shot start (XINIT for the CRC,
// 0 for the polynomials), so the chunk's state is carried over it here:
// CRC32_ex(d, X) = FINAL-form crc ^ ~0 ^ M^|d| (X ^ ~0) and
// h(d, X) = M^|d| X + h(d, 0) for simple_hash / Time33 (orders divide 2^30).
__global__ void big_patch_state_kernel(const uint32_t *__restrict__ nbig, const uint32_t *__restrict__ order,
                                       uint32_t n, const uint32_t *__restrict__ bcrc, const uint32_t *__restrict__ bpoly,
                                       const uint64_t *__restrict__ sizes, const uint32_t *__restrict__ sidx,
                                       bool md5, fdfs_gpu_file_state *__restrict__ states,
                                       const DevTables *__restrict__ tabs)
{
    const uint32_t nb = *nbig;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += gridDim.x * blockDim.x) {
        const uint32_t f = order[i];
        if (f >= n)  // flagged by big_plan_kernel
            continue;
        const uint64_t L = sizes[f];
        fdfs_gpu_file_state *fs = states + (sidx ? sidx[f] : f);
        const uint32_t c = bcrc[i] ^ 0xFFFFFFFFu ^ advance_bytes(tabs->t, ~(uint32_t)fs->crc32, L);
        if (md5) {
            fs->crc32 = (int32_t)c;
            continue;
        }
        const uint32_t e = (uint32_t)(L & 0x3FFFFFFFull);
        const uint32_t s = pow_dev(31u, e) * (uint32_t)fs->hash_codes[2] + bpoly[2ull * i];
        const uint32_t t = pow_dev(33u, e) * (uint32_t)fs->hash_codes[3] + bpoly[2ull * i + 1];
        fs->crc32 = (int32_t)c;
        fs->hash_codes[0] = (int32_t)c;
        fs->hash_codes[2] = (int32_t)s;
        fs->hash_codes[3] = (int32_t)t;
    }
}

// ------------------------------------------------------------------ launchers

// Zeroing as a kernel rather than hipMemsetAsync: inside a captured hipGraph
// a kernel node is ordered like every other node of the chain, and the lane
// path's size histogram must be zero before bin_hist_kernel counts into it.
__global__ void zero_u32_kernel(uint32_t *__restrict__ p, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = 0;
}

hipError_t launch_zero_u32(void *p, uint64_t ndwords, hipStream_t st)
{
    if (ndwords == 0)
        return hipSuccess;
    uint64_t g = (ndwords + 255) / 256;
    zero_u32_kernel<<<(unsigned)(g < 4096 ? g : 4096), 256, 0, st>>>(static_cast<uint32_t *>(p), ndwords);
    return hipGetLastError();
}

// The context's lane-path error count (fdfs_api.cpp lane_err_note): +1 when
// this launch's error word is set (word == nullptr: a fault injected by
// fdfs_gpu_inject_error).  A context may be called on several streams, so
// two of these can run at once: the add is a device-scope atomic, and the
// new count goes to the launch's own host slot (fdfs_api.cpp lane_err_note).
__global__ void lane_err_count_kernel(const uint32_t *__restrict__ word, unsigned long long *__restrict__ count,
                                      unsigned long long *__restrict__ slot)
{
    if (threadIdx.x == 0) {
        const unsigned long long inc = (!word || *word) ? 1ull : 0ull;
        *slot = atomicAdd(count, inc) + inc;
    }
}

hipError_t launch_lane_err_count(const uint32_t *word, uint64_t *count, uint64_t *slot, hipStream_t st)
{
    lane_err_count_kernel<<<1, 64, 0, st>>>(word, reinterpret_cast<unsigned long long *>(count),
                                            reinterpret_cast<unsigned long long *>(slot));
    return hipGetLastError();
}

// Small scans (a batch's segment counts, a small dedup's [digit][tile]
// counts) in one block: one launch instead of three.  Only up to one pass of
// the block: a single CU moves the 63K counts of a 1M-record dedup in 38 us
// against 21 us for the three-kernel form (profiles/r02/scan_kernels.txt).
constexpr int kScan1Items = 16;
constexpr uint64_t kScan1Max = 1024ull * kScan1Items;

__global__ __launch_bounds__(1024) void scan_single_kernel(const uint64_t *__restrict__ in, uint64_t n,
                                                           uint64_t *__restrict__ out)
{
    __shared__ uint64_t wsum[1024 / 64];
    uint64_t carry = 0;
    for (uint64_t c0 = 0; c0 < n; c0 += 1024 * kScan1Items) {
        const uint64_t b0 = c0 + (uint64_t)threadIdx.x * kScan1Items;
        // branch-free loads (clamped index, masked value): all of a thread's
        // loads leave together instead of one round trip per item
        uint64_t vals[kScan1Items];
        uint64_t v = 0;
#pragma unroll
        for (int k = 0; k < kScan1Items; k++)
            vals[k] = in[b0 + k < n ? b0 + k : n - 1];
#pragma unroll
        for (int k = 0; k < kScan1Items; k++) {
            vals[k] = (b0 + k < n) ? vals[k] : 0;
            v += vals[k];
        }
        uint64_t tot;
        uint64_t run = carry + block_exclusive_scan(v, wsum, tot);
#pragma unroll
        for (int k = 0; k < kScan1Items; k++) {
            if (b0 + k < n)
                out[b0 + k] = run;
            run += vals[k];
        }
        carry += tot;
    }
    if (threadIdx.x == 0)
        out[n] = carry;
}

hipError_t launch_exclusive_scan(const uint64_t *in, uint64_t n, uint64_t *out, uint64_t *bsum,
                                 hipStream_t st)
{
    if (n == 0)
        return launch_zero_u32(out, 2, st);
    if (n <= kScan1Max) {
        scan_single_kernel<<<1, 1024, 0, st>>>(in, n, out);
        return hipGetLastError();
    }
    const uint64_t nb = (n + kScanTile - 1) / kScanTile;
    scan_reduce_kernel<<<(unsigned)nb, kScanBlock, 0, st>>>(in, n, bsum);
    scan_sums_kernel<<<1, 1024, 0, st>>>(bsum, nb);
    scan_apply_kernel<<<(unsigned)nb, kScanBlock, 0, st>>>(in, n, bsum, out);
    return hipGetLastError();
}

uint64_t scan_workspace_elems(uint64_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

static hipError_t crc_seg_run(bool sar, const uint8_t *base, const uint64_t *offs, const uint64_t *sizes,
                              const uint64_t *seg_first, uint32_t n, const uint32_t *n_dev,
                              const DevTables *tabs, uint32_t *crc_out, unsigned ncu, hipStream_t st);

hipError_t launch_sig_lane(bool sar, int method, const uint8_t *base, const uint64_t *offs,
                           const uint64_t *sizes, uint32_t n, uint32_t *hist, uint32_t *order,
                           const BigCrcWs *big, const DevTables *tabs, uint32_t *crc_out,
                           uint8_t *sig_out, int32_t *codes_out, fdfs_gpu_file_state *states,
                           const uint32_t *sidx, unsigned ncu, hipStream_t st,
                           hipEvent_t ev0, hipEvent_t ev1)
{
    if (method == 0 && (states || big == nullptr))
        return hipErrorInvalidValue;  // the CRC-only lane path is one-shot, big files offloaded
    hipError_t e = launch_zero_u32(hist, kLaneWsDwords, st);
    if (e != hipSuccess)
        return e;
    uint32_t *cursor = hist + kSizeBins;
    const unsigned hb = (n + 1023) / 1024, sb = (n + 1024 * kBinItems - 1) / (1024 * kBinItems);
    // bmask: the bins' low mantissa bits cleared (all kept: 1/32-octave
    // bins; merging 2^s of them measured slower)
    const uint32_t bmask = ~0u;
    bin_hist_kernel<<<hb < 128 ? hb : 128, 1024, 0, st>>>(sizes, n, hist, bmask);
    bin_scan_kernel<<<1, 1024, 0, st>>>(hist, cursor);
    uint32_t *err = hist + kLaneErrWord;
    bin_scatter_kernel<<<sb, 1024, 0, st>>>(sizes, n, cursor, order, err, bmask);
    const bool offload = big != nullptr;
    if (ev0 && method == 0)  // CRC only: the events cover the fold of the big files too
        (void)hipEventRecord(ev0, st);
    if (offload) {
        // the segmented passes over the files >= T (CRC; HASH: simple_hash,
        // Time33 too), before the lane kernel (beside it on a second stream
        // measured no faster: the two compete for HBM)
        big_plan_kernel<<<1, 1024, 0, st>>>(hist, order, offs, sizes, n, method, big->lat_files, big->nbig,
                                            big->big_min, big->offs, big->sizes, big->seg_first, big->crc, big->poly,
                                            err);
        if ((e = crc_seg_run(sar, base, big->offs, big->sizes, big->seg_first, n, big->nbig, tabs, big->crc,
                             big->ncu, st)) != hipSuccess)
            return e;
        // poly_seg_kernel: 2 workgroups of 4 waves per CU (its own grid; the
        // CRC kernel's is one 8-wave workgroup per CU)
        if (method == 1 && (e = launch_poly_seg(base, big->offs, big->sizes, big->seg_first, big->nbig, big->poly,
                                                2 * big->ncu, st)) != hipSuccess)
            return e;
    }
    const uint64_t *bmin = offload ? big->big_min : nullptr;
    if (ev0 && method != 0)
        (void)hipEventRecord(ev0, st);
    // HASH batches (big files >= T: big_plan_kernel's adaptive T up to
    // lat_files files, kBigCrcMin above) and MD5 batches small enough to
    // offload (n <= lat_files), one-shot or chunked: when there are at most
    // one big file per CU each runs its serial chain (ELF / MD5) on a
    // workgroup of its own; MD5 up to one per SIMD on a wave of its own (the
    // ELF form of that, probes/extra/chain_wave.patch, gains 6 % at 1,024
    // uploads per call and is kept out of sig_hash_kernel, the headline
    // kernel: profiles/r06/chain_wave_ab.txt)
    const bool chains = offload && (method == 1 || (method == 2 && n <= big->lat_files));
    e = (method == 2)   ? launch_md5_stage(sar, base, offs, sizes, n, order, tabs, bmin, hist + 2 * kSizeBins,
                                           crc_out, sig_out, codes_out, states, sidx, big ? big->ncu : 0, st,
                                           chains ? big->nbig : nullptr, chains ? 4 * big->ncu : 0u)
        : (method == 1) ? launch_sig_hash(sar, base, offs, sizes, n, order, tabs, bmin, crc_out, sig_out,
                                          codes_out, states, sidx, st, chains ? big->nbig : nullptr,
                                          chains ? big->ncu : 0u)
                        : launch_crc_lane(sar, base, offs, sizes, n, order, tabs, bmin, crc_out, st);
    if (e != hipSuccess)
        return e;
    if (ev1)
        (void)hipEventRecord(ev1, st);
    if (offload && states)
        big_patch_state_kernel<<<256, 256, 0, st>>>(big->nbig, order, n, big->crc, big->poly, sizes, sidx,
                                                    method == 2, states, tabs);
    else if (offload)
        big_patch_kernel<<<256, 256, 0, st>>>(big->nbig, order, n, big->crc, big->poly, method == 2,
                                              crc_out, sig_out, codes_out);
    return hipGetLastError();
}

static hipError_t crc_seg_run(bool sar, const uint8_t *base, const uint64_t *offs, const uint64_t *sizes,
                              const uint64_t *seg_first, uint32_t n, const uint32_t *n_dev,
                              const DevTables *tabs, uint32_t *crc_out, unsigned ncu, hipStream_t st)
{
    static const int bpc = crc_seg_blocks_per_cu();
    const unsigned grid = ncu * (unsigned)bpc;
    if (sar)
        crc_seg_kernel<true><<<grid, kSegBlock, kSegRingBytes, st>>>(base, offs, sizes, seg_first, n, n_dev, tabs, crc_out);
    else
        crc_seg_kernel<false><<<grid, kSegBlock, kSegRingBytes, st>>>(base, offs, sizes, seg_first, n, n_dev, tabs, crc_out);
    return hipGetLastError();
}

static hipError_t crc_tab_run(bool sar, const uint8_t *base, const uint64_t *offs, const uint64_t *sizes,
                              const uint64_t *seg_first, uint32_t n, const DevTables *tabs, uint32_t *crc_out,
                              unsigned ncu, hipStream_t st)
{
    static const int bpc = crc_tab_blocks_per_cu();
    const unsigned grid = ncu * (unsigned)bpc;
    if (sar)
        crc_tab_kernel<true><<<grid, kSegBlock, 0, st>>>(base, offs, sizes, seg_first, n, nullptr, tabs, crc_out);
    else
        crc_tab_kernel<false><<<grid, kSegBlock, 0, st>>>(base, offs, sizes, seg_first, n, nullptr, tabs, crc_out);
    return hipGetLastError();
}

hipError_t launch_crc_seg(bool sar, const uint8_t *base, const uint64_t *offs, const uint64_t *sizes,
                          uint32_t n, uint64_t *nseg, uint64_t *seg_first, uint64_t *bsum,
                          const DevTables *tabs, uint32_t *crc_out, unsigned ncu, hipStream_t st,
                          hipEvent_t ev0, hipEvent_t ev1)
{
    hipError_t e;
    uint64_t *first_tab = seg_first, *first_fold = seg_first + (size_t)n + 1;
    if (n < kPlanSmall) {
        plan_small_kernel<<<1, 1024, 0, st>>>(sizes, n, seg_first, crc_out);
    } else {
        plan_nseg_kernel<<<(n + 255) / 256, 256, 0, st>>>(sizes, n, nseg, crc_out);
        if ((e = launch_exclusive_scan(nseg, n, first_tab, bsum, st)) != hipSuccess ||
            (e = launch_exclusive_scan(nseg + n, n, first_fold, bsum + scan_workspace_elems(n), st)) != hipSuccess)
            return e;
    }
    if (ev0)
        (void)hipEventRecord(ev0, st);
    if ((e = crc_tab_run(sar, base, offs, sizes, first_tab, n, tabs, crc_out, ncu, st)) != hipSuccess ||
        (e = crc_seg_run(sar, base, offs, sizes, first_fold, n, nullptr, tabs, crc_out, ncu, st)) != hipSuccess)
        return e;
    if (ev1)
        (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

int crc_seg_blocks_per_cu()
{
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, crc_seg_kernel<true>, kSegBlock, kSegRingBytes) != hipSuccess)
        return 1;
    return nb > 0 ? nb : 1;
}

int crc_tab_blocks_per_cu()
{
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, crc_tab_kernel<true>, kSegBlock, 0) != hipSuccess)
        return 1;
    return nb > 0 ? nb : 1;
}

}  // namespace fdfs
