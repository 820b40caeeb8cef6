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
//  * dedup_group: partition, then group each partition in LDS.
//      K1 dp_tile      key32 = low half of a 64-bit mix of the signature;
//                      each 8192-record tile sorted by the top D1 bits in LDS
//                      and written back contiguously
//      K2 scan         exclusive scan of the [digit][tile] counts
//      K3 chunks       D1 buckets cut into 8192-entry chunks
//      K4 dp_split     one workgroup per chunk: gathers its entries along the
//                      tile runs, sorts them by the next D2 bits in LDS and
//                      writes the chunk back contiguously
//      K5 dp_group     one workgroup per partition (~1.5K records): gathers
//                      its run from each chunk of its bucket; an
//                      open-addressing table in LDS keyed by key bits, a
//                      slot is claimed by 32-bit CAS of {key bits, claimer's
//                      local index} and never changes, the entries that met
//                      an equal key are listed and confirmed on the full 24
//                      bytes against the claimer's row, class min(gidx) and
//                      size by LDS atomics, then rep/ref written per record
//                      of a multi-member class.
//    Every random-access atomic stays in LDS: device-scope atomics to
//    random addresses run at a few percent of the HBM rate on MI355X
//    (MI355X_MICROARCH.md, global atomics), which is what bounded the
//    single global hash table this replaces (20 ms for 100M records).
//    A partition with more records than the LDS table holds (heavy
//    duplication of one signature, or adversarial keys) is grouped by the
//    same code on a table in HBM, in a region of the workspace that belongs
//    to that partition alone; results do not depend on arrival order.
#include "fdfs_device.hpp"
#include "fdfs_kernels.hpp"

#include <climits>
#include <cstdlib>
#include <type_traits>

namespace fdfs {

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

__device__ __forceinline__ bool sig_equal(const uint8_t *sig, uint32_t stride, uint32_t x, uint32_t y)
{
    uint64_t a, b, c, a2, b2, c2;
    load_sig(sig + (uint64_t)x * stride, a, b, c);
    load_sig(sig + (uint64_t)y * stride, a2, b2, c2);
    return a == a2 && b == b2 && c == c2;
}

// Partition plan.  Entries are 8 bytes, {key32 << 32 | record}; a record's
// partition is the top d1 + d2 bits of key32 (~1K records per partition).
//  K1 dp_tile   a tile of kDpTile records: keys, singleton answers, the tile's
//               entries sorted by the top d1 bits in LDS and written back
//               contiguously (one coalesced run per tile, no scatter);
//               per (digit, tile) count and in-tile start
//  K2 scan      exclusive scan of the [digit][tile] counts: where each tile's
//               run of a digit goes in the bucket-sorted order
//  K3 chunks    each d1 bucket cut into kDpChunk-entry chunks (positions in
//               the bucket-sorted order); the tile holding each chunk's
//               first position
//  K4 dp_split  one workgroup per chunk: gathers the chunk's entries from the
//               tile runs (coalesced reads along each run), sorts them by the
//               next d2 bits in LDS, writes the chunk back contiguously and
//               the chunk's d2 digit starts (u16)
//  K5 dp_group  one workgroup per partition (bucket b, digit d): gathers its
//               run from each chunk of bucket b, then groups in LDS
// Every HBM write of K1 and K4 is a whole contiguous tile/chunk (round 1's
// scatter and split wrote ~16-entry runs per digit: partial lines, 1.2x
// their bytes), and the split needs no counting pass.
constexpr int kDpTileThreads = 512;
constexpr int kDpTileItems = 16;
constexpr int kDpTile = kDpTileThreads * kDpTileItems;  // records per K1 tile
constexpr int kDpMaxD1 = 8;
constexpr int kDpMaxD2 = 12;
constexpr int kDpSplitThreads = 1024;
constexpr int kDpSplitPer = 8;
constexpr int kDpChunk = kDpSplitThreads * kDpSplitPer;  // entries per K4 chunk
static_assert(kDpChunk < 65536, "chunk digit starts are u16");
// The group kernel is latency-bound: a partition is a chain of dependent
// round trips (run table, entries, confirmation rows, answers), so its rate
// is the number of records in flight per CU, which LDS and registers cap.
// Round 3: 512-thread workgroups of up to 2048 records (four entries per
// thread, mean <= 1536), an LDS table of 32-bit words {key bits, local
// index} (the partition's records by local index beside it), and only the
// entries that met an equal key -- compacted into a list -- load rows, so
// no thread holds rows for entries that joined nothing.  40 KB per
// workgroup (GM_INDEX; 48 KB with 64-bit class minima): four workgroups =
// 8192 records in flight per CU, twice round 2's two-entry form (64-bit
// words {key32, record}, 20 B per slot at two slots per record).
constexpr int kDpGroupThreads = 512;
constexpr int kDpEpt = 4;  // entries per thread
constexpr uint32_t kDpCap = kDpGroupThreads * kDpEpt;  // records per partition grouped in LDS
// 3070 slots: load <= 2/3 at the cap (<= 1/2 at dp_plan's mean); the two
// spare words of a 3072-word region keep the arrays after it 8-byte aligned.
constexpr uint32_t kDpSlots = kDpCap * 3 / 2 - 2;
constexpr int kDpLocBits = 12;  // local index field of an LDS table word
static_assert(kDpCap < (1u << kDpLocBits), "local index field");
constexpr uint32_t kDpKeyMask = (1u << (32 - kDpLocBits)) - 1;  // key bits kept in a word
constexpr uint32_t kDpWEmpty = ~0u;
constexpr uint64_t kDpEmpty = ~0ull;
constexpr int kDpRuns = kDpGroupThreads;  // chunk runs per K5 gather batch (one per thread)

struct DpPlan {
    int d1, d2;          // partition bits: top d1 of key32 (K1), next d2 (K4)
    uint64_t tiles;      // K1 tiles
    uint64_t chunks;     // bound on K4 chunks: sum over buckets of ceil(size / kDpChunk)
    uint64_t nparts() const { return 1ull << (d1 + d2); }
    uint64_t ncnt() const { return (1ull << d1) * tiles; }
};

DpPlan dp_plan(uint64_t n)
{
    int p = 1;  // partitions of mean n / 2^p <= 3/4 of kDpCap
    while (p < kDpMaxD1 + kDpMaxD2 && (n >> p) > kDpCap / 4 * 3)
        p++;
    DpPlan pl;
    pl.d1 = p < kDpMaxD1 ? p : kDpMaxD1;
    pl.d2 = p - pl.d1;
    pl.tiles = (n + kDpTile - 1) / kDpTile;
    pl.chunks = (n + kDpChunk - 1) / kDpChunk + (1ull << pl.d1);
    return pl;
}

// Exclusive scan of cnt[0, nb) into out[] by the whole block (each thread
// owns PER consecutive bins; nb <= PER * blockDim.x).
template <int PER, int NT>
__device__ __forceinline__ void block_scan_bins(const uint32_t *cnt, uint32_t *out, uint32_t nb,
                                                uint32_t *wsum)
{
    uint32_t v[PER], sum = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const uint32_t k = threadIdx.x * PER + q;
        v[q] = k < nb ? cnt[k] : 0u;
        sum += v[q];
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o)
            x += y;
    }
    if (lane == 63)
        wsum[wid] = x;
    __syncthreads();
    uint32_t run = x - sum;
    for (int k = 0; k < wid; k++)
        run += wsum[k];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const uint32_t k = threadIdx.x * PER + q;
        if (k < nb)
            out[k] = run;
        run += v[q];
    }
    __syncthreads();
}

// One value per thread: exclusive prefix over the block and the block total.
__device__ __forceinline__ uint32_t block_scan1(uint32_t v, uint32_t *wsum, uint32_t &total)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o)
            x += y;
    }
    if (lane == 63)
        wsum[wid] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); k++) {
        if (k < wid)
            pre += wsum[k];
        tot += wsum[k];
    }
    __syncthreads();
    total = tot;
    return pre + x - v;
}

__device__ __forceinline__ uint64_t block_exclusive_scan64(uint64_t v, uint64_t *wsum, uint64_t &total)
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

// Max over the threads before this one (-1 for thread 0).
__device__ __forceinline__ int32_t block_max_excl(int32_t v, int32_t *wmax)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o);
        if (lane >= o)
            x = y > x ? y : x;
    }
    if (lane == 63)
        wmax[wid] = x;
    __syncthreads();
    int32_t run = __shfl_up(x, 1);
    if (lane == 0)
        run = -1;
    for (int k = 0; k < wid; k++)
        run = wmax[k] > run ? wmax[k] : run;
    __syncthreads();
    return run;
}

// Per-record answers: two arrays (rep u64[n], ref u32[n]), or packed (the
// fdfs_gpu_dedup_answer array of fdfs_gpu_dedup_packed, and the exchange
// rows of fdfs_gpu_dedup_global): 16 bytes {rep, ref, 0} per record at
// `rep`.  Packed, a record's two answers share a line: one random store in
// dp_group instead of two.
struct DpOut {
    uint64_t *rep;
    uint32_t *ref;
    bool packed;
    __device__ __forceinline__ uint64_t rep_at(uint64_t r) const { return packed ? rep[2 * r] : rep[r]; }
    __device__ __forceinline__ void store(uint64_t r, uint64_t rp, uint32_t rf, bool with_rep) const
    {
        if (packed) {
            *reinterpret_cast<uint4 *>(rep + 2 * r) = make_uint4((uint32_t)rp, (uint32_t)(rp >> 32), rf, 0u);
        } else {
            if (with_rep)
                rep[r] = rp;
            ref[r] = rf;
        }
    }
};

// The owner side of fdfs_gpu_dedup_global (round 6): only the records of
// multi-member classes are answered, as 16-byte records {sender row, ref,
// rep lo, rep hi} appended per segment of the owner's rows (one segment per
// sending rank, seg_start[k] .. seg_start[k + 1]; the sender pre-filled
// every record's singleton answer in its bucket pass).  With the bench's 10 %
// duplicates ~20 % of the rows are answered, so the way back carries ~0.2x
// the bytes of an answer per row.  Segment k's records go to ans[seg_start[k]
// + slot] (room for every row of the segment), slot from cntr[k]: one
// device-scope atomic per (workgroup, segment) after an LDS count.
struct DpSink {
    uint4 *ans;              // null: answers go to DpOut (the one-GPU forms)
    uint32_t *cntr;          // [nseg] records appended per segment
    const uint64_t *seg;     // seg_start[0 .. nseg], then seg_soff[0 .. nseg - 1] at seg + kSinkSoff
    uint32_t nseg;
    // the segment holding owner row `row` (nseg <= 64: a uniform scan)
    __device__ __forceinline__ uint32_t seg_of(uint64_t row) const
    {
        uint32_t s = 0;
        for (uint32_t k = 1; k < nseg; k++)
            s += row >= seg[k] ? 1u : 0u;
        return s;
    }
    __device__ __forceinline__ void put(uint32_t s, uint32_t slot, uint64_t row, uint64_t rep, uint32_t ref) const
    {
        const uint32_t src = (uint32_t)(seg[kSinkSoff + s] + (row - seg[s]));  // the sender's row
        ans[seg[s] + slot] = make_uint4(src, ref, (uint32_t)rep, (uint32_t)(rep >> 32));
    }
};

// K1: keys, the singleton answer (rep = own gidx, ref = 1) of every record,
// and the tile's entries sorted by digit (top d1 bits; unstable: order inside
// a partition does not matter) written back as one contiguous run.  With a
// DpSink (out.rep null) no singleton answer is written here: the senders
// wrote them.
__global__ __launch_bounds__(kDpTileThreads) void dp_tile_kernel(
    const uint8_t *__restrict__ sig, uint32_t stride, const uint64_t *__restrict__ gidx,
    uint32_t gstride, uint64_t n, int d1, uint64_t tiles, uint64_t *__restrict__ ent1,
    DpOut out, uint64_t *__restrict__ cnt1,
    uint32_t *__restrict__ loc1)
{
    __shared__ uint32_t h[1 << kDpMaxD1];
    __shared__ uint32_t lst[1 << kDpMaxD1];
    __shared__ uint32_t wsum[kDpTileThreads / 64];
    __shared__ uint64_t stage[kDpTile];
    const uint32_t nb = 1u << d1;
    for (uint32_t k = threadIdx.x; k < nb; k += blockDim.x)
        h[k] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kDpTile;
    const uint32_t m = (uint32_t)((n - t0) < (uint64_t)kDpTile ? (n - t0) : (uint64_t)kDpTile);
    uint32_t key[kDpTileItems], rank[kDpTileItems];
#pragma unroll
    for (int it = 0; it < kDpTileItems; it++) {
        const uint32_t l = it * kDpTileThreads + threadIdx.x;
        if (l < m) {
            const uint64_t r = t0 + l;
            uint64_t a, b, c;
            load_sig(sig + r * stride, a, b, c);
            key[it] = (uint32_t)sig_hash(a, b, c);
            // every record starts as its own class; dp_group overwrites the
            // records of classes with more than one member (writing these
            // from dp_split instead measured neutral)
            if (out.rep)
                out.store(r, gstride ? gidx[r * gstride] : r, 1u, true);
        }
    }
#pragma unroll
    for (int it = 0; it < kDpTileItems; it++) {
        const uint32_t l = it * kDpTileThreads + threadIdx.x;
        if (l < m)
            rank[it] = atomicAdd(&h[key[it] >> (32 - d1)], 1u);
    }
    __syncthreads();
    block_scan_bins<1, kDpTileThreads>(h, lst, nb, wsum);
#pragma unroll
    for (int it = 0; it < kDpTileItems; it++) {
        const uint32_t l = it * kDpTileThreads + threadIdx.x;
        if (l < m)
            stage[lst[key[it] >> (32 - d1)] + rank[it]] = ((uint64_t)key[it] << 32) | (uint32_t)(t0 + l);
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < m; j += blockDim.x)
        ent1[t0 + j] = stage[j];
    for (uint32_t k = threadIdx.x; k < nb; k += blockDim.x) {
        cnt1[(uint64_t)k * tiles + blockIdx.x] = h[k];
        loc1[(uint64_t)k * tiles + blockIdx.x] = lst[k];
    }
}

// K3a: chunks per bucket, exclusive prefix -> cb[0..nb1] (one block of 256).
__global__ __launch_bounds__(256) void dp_chunks_kernel(const uint64_t *__restrict__ off1, int d1,
                                                        uint64_t tiles, uint32_t *__restrict__ cb,
                                                        uint32_t *__restrict__ slow)
{
    if (threadIdx.x == 0)
        slow[0] = 0;  // K5's list of partitions for dp_group_slow_kernel
    __shared__ uint32_t c[1 << kDpMaxD1];
    __shared__ uint32_t s[1 << kDpMaxD1];
    __shared__ uint32_t wsum[4];
    const uint32_t nb1 = 1u << d1;
    for (uint32_t k = threadIdx.x; k < nb1; k += blockDim.x) {
        const uint64_t size = off1[(uint64_t)(k + 1) * tiles] - off1[(uint64_t)k * tiles];
        c[k] = (uint32_t)((size + kDpChunk - 1) / kDpChunk);
    }
    __syncthreads();
    block_scan_bins<1, 256>(c, s, nb1, wsum);
    for (uint32_t k = threadIdx.x; k < nb1; k += blockDim.x)
        cb[k] = s[k];
    if (threadIdx.x == 0)
        cb[nb1] = s[nb1 - 1] + c[nb1 - 1];
}

// K3b: for every non-empty (digit, tile) run, the chunks of that bucket whose
// first position falls inside it start at that tile.
// Each chunk also gets its descriptor {P0 lo, P0 hi, m, b | last << 31}
// (first position, entry count, bucket, last chunk of its bucket), so that
// dp_split starts with one round of independent loads.
__global__ void dp_chunk_ta_kernel(const uint64_t *__restrict__ off1, uint64_t tiles, uint64_t ncnt,
                                   const uint32_t *__restrict__ cb, uint32_t *__restrict__ chunk_ta,
                                   uint4 *__restrict__ chunk_hd)
{
    for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < ncnt;
         idx += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t o = off1[idx], o2 = off1[idx + 1];
        if (o2 <= o)
            continue;
        const uint64_t b = idx / tiles, t = idx - b * tiles;
        const uint64_t bs = off1[b * tiles], be = off1[(b + 1) * tiles];
        for (uint64_t k = (o - bs + kDpChunk - 1) / kDpChunk; bs + k * kDpChunk < o2; k++) {
            const uint64_t P0 = bs + k * kDpChunk;
            const uint64_t m = be - P0 < (uint64_t)kDpChunk ? be - P0 : (uint64_t)kDpChunk;
            const uint32_t last = P0 + kDpChunk >= be ? 1u : 0u;
            chunk_ta[cb[b] + k] = (uint32_t)t;
            chunk_hd[cb[b] + k] = make_uint4((uint32_t)P0, (uint32_t)(P0 >> 32), (uint32_t)m, (uint32_t)b | last << 31);
        }
    }
}

// K4: one workgroup per chunk (global chunk id g; bucket b = the one with
// cb[b] <= g < cb[b + 1]).  Every position of the chunk is mapped to its
// source in the tile-sorted K1 output: each tile run overlapping the chunk
// marks its first position with (source - position), a block max-scan carries
// the mark over the run, and the entries are loaded along the runs.  They are
// then ranked by the d2 digit in LDS and the chunk goes back contiguously.
constexpr int64_t kDpNoMark = INT64_MIN;

// The position -> source buffer is stored swizzled: position i at
// dp_sw(i), which permutes the 16-byte pairs inside each 64-byte row of 8
// positions by bits 4-5 of i.  The max-scan reads a thread's own row with
// 16-byte loads at a 64-byte stride; unswizzled, those rows land on the same
// banks for every other lane (before: 119M of 177M LDS-active cycles were
// bank conflicts, profiles/r03/dedup_pmc.txt), swizzled the 8 lanes of each
// 128-byte LDS pass hit 8 distinct 16-byte bank groups.  Position-order
// accesses (lane l at position base + l) stay conflict-free: the
// permutation does not leave a row.
__device__ __forceinline__ uint32_t dp_sw(uint32_t i) { return i ^ (((i >> 4) & 3u) << 1); }

// NB: digit bins (1 << d2 <= NB); 1024 bins keep the LDS at 72 KB, two
// workgroups per CU.
template <int NB>
__global__ __launch_bounds__(kDpSplitThreads) void dp_split_kernel(
    const uint64_t *__restrict__ ent1, int d1, int d2, uint64_t tiles, const uint64_t *__restrict__ off1,
    const uint32_t *__restrict__ loc1, const uint32_t *__restrict__ cb, const uint32_t *__restrict__ chunk_ta,
    const uint4 *__restrict__ chunk_hd, uint64_t *__restrict__ ent2, uint16_t *__restrict__ cdo,
    DpOut out, const uint64_t *__restrict__ gidx, uint32_t gstride, uint64_t n)
{
    constexpr int NT = kDpSplitThreads;
    constexpr int PER = NB / NT;
    static_assert(NB % NT == 0, "bins per thread");
    static_assert(kDpSplitPer == 8, "one 64-byte row of positions per thread");
    __shared__ int64_t buf[kDpChunk];  // position -> source offset (swizzled), then the digit-sorted chunk
    __shared__ uint32_t cc[NB];        // chunk digit counts
    __shared__ uint32_t cl[NB];        // chunk digit starts
    __shared__ uint32_t wsum[NT / 64];
    __shared__ int32_t wmax[NT / 64];
    const uint32_t nb1 = 1u << d1, nd2 = 1u << d2;
    const uint32_t g = blockIdx.x;
    // one round of independent loads: the chunk count, this chunk's
    // descriptor and tile range (read before the bound check; unused past it)
    const uint32_t nch = cb[nb1];
    const uint4 hd = chunk_hd[g];
    const uint32_t ta = chunk_ta[g], tn = chunk_ta[g + 1 < gridDim.x ? g + 1 : g];
    if (g >= nch)  // past the last chunk (the grid is a bound)
        return;
    const uint32_t b = hd.w & 0x7FFFFFFFu;
    const uint64_t P0 = (uint64_t)hd.x | (uint64_t)hd.y << 32;
    const uint32_t m = hd.z;
    const uint32_t tb = (hd.w >> 31) ? (uint32_t)(tiles - 1) : tn;
    const uint64_t *ob = off1 + (uint64_t)b * tiles;
    const uint32_t *lb = loc1 + (uint64_t)b * tiles;
    for (uint32_t k = threadIdx.x; k < nd2; k += NT)
        cc[k] = 0;
    for (uint32_t i = threadIdx.x; i < m; i += NT)
        buf[dp_sw(i)] = kDpNoMark;
    __syncthreads();
    for (uint32_t t = ta + threadIdx.x; t <= tb; t += NT) {
        const uint64_t o = ob[t], o2 = ob[t + 1];
        const uint64_t lo = o > P0 ? o : P0;
        const uint64_t hi = o2 < P0 + m ? o2 : P0 + m;
        if (lo < hi)
            buf[dp_sw((uint32_t)(lo - P0))] = (int64_t)((uint64_t)t * kDpTile + lb[t]) - (int64_t)o;
    }
    __syncthreads();
    // carry each mark over its run: thread owns positions [i0, i0 + 8), one
    // row, read as four 16-byte pairs (pair j of the row sits at j ^ sw)
    const uint32_t i0 = threadIdx.x * kDpSplitPer;
    const uint32_t sw = (threadIdx.x >> 1) & 3u;
    uint4 *bufv = reinterpret_cast<uint4 *>(buf);
    int64_t bv[kDpSplitPer];
#pragma unroll
    for (int j = 0; j < kDpSplitPer / 2; j++) {
        const uint4 v = bufv[threadIdx.x * 4 + (j ^ sw)];
        bv[2 * j] = (int64_t)((uint64_t)v.x | (uint64_t)v.y << 32);
        bv[2 * j + 1] = (int64_t)((uint64_t)v.z | (uint64_t)v.w << 32);
    }
    int32_t lp = -1;
#pragma unroll
    for (int q = 0; q < kDpSplitPer; q++)
        if (i0 + q < m && bv[q] != kDpNoMark)
            lp = (int32_t)(i0 + q);
    const int32_t cur = block_max_excl(lp, wmax);
    // the mark carried in from the threads before (position 0 is always
    // marked, chunk_ta), then this row's own marks
    int64_t val = cur >= 0 ? buf[dp_sw((uint32_t)cur)] : 0;
#pragma unroll
    for (int q = 0; q < kDpSplitPer; q++) {
        if (bv[q] != kDpNoMark)
            val = bv[q];
        bv[q] = val;  // positions >= m: unused
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kDpSplitPer / 2; j++)
        bufv[threadIdx.x * 4 + (j ^ sw)] =
            make_uint4((uint32_t)bv[2 * j], (uint32_t)((uint64_t)bv[2 * j] >> 32), (uint32_t)bv[2 * j + 1],
                       (uint32_t)((uint64_t)bv[2 * j + 1] >> 32));
    __syncthreads();
    const int sh = 64 - d1 - d2;  // d2 digit = (entry >> sh) & (nd2 - 1)
    uint64_t en[kDpSplitPer];
    uint32_t rk[kDpSplitPer];
#pragma unroll
    for (int q = 0; q < kDpSplitPer; q++) {
        const uint32_t l = q * NT + threadIdx.x;
        if (l < m)
            en[q] = ent1[(uint64_t)(buf[dp_sw(l)] + (int64_t)(P0 + l))];
    }
#pragma unroll
    for (int q = 0; q < kDpSplitPer; q++) {
        const uint32_t l = q * NT + threadIdx.x;
        if (l < m)
            rk[q] = atomicAdd(&cc[(uint32_t)(en[q] >> sh) & (nd2 - 1)], 1u);
    }
    __syncthreads();
    block_scan_bins<PER, NT>(cc, cl, nd2, wsum);
    uint64_t *stage = reinterpret_cast<uint64_t *>(buf);
#pragma unroll
    for (int q = 0; q < kDpSplitPer; q++) {
        const uint32_t l = q * NT + threadIdx.x;
        if (l < m)
            stage[cl[(uint32_t)(en[q] >> sh) & (nd2 - 1)] + rk[q]] = en[q];
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < m; j += NT)
        ent2[P0 + j] = stage[j];
    for (uint32_t k = threadIdx.x; k < nd2; k += NT)
        cdo[(uint64_t)g * nd2 + k] = (uint16_t)cl[k];
}

// Open-addressing tables, linear probing from a multiplicative home slot.
// Every slot is set once by CAS and never changed, so the first slot with a
// given key along a probe sequence is the same for every later probe.
__device__ __forceinline__ uint32_t dp_home(uint32_t key, uint32_t size)
{
    return (uint32_t)(((uint64_t)(key * 0x9E3779B1u) * size) >> 32);
}

__device__ __forceinline__ uint32_t dp_next(uint32_t slot, uint32_t size)
{
    return slot + 1 == size ? 0 : slot + 1;
}

// HBM table of an oversized partition: 64-bit words {key32, claimer record}.
// Key-only probe from `slot`: claim the first empty slot, or stop at the
// first slot whose key equals ours.  Returns the slot; `owner` = its claimer
// (r itself when this record claimed it).  Equal keys still need the
// full-signature check (dp_insert continues past a mismatch).
__device__ __forceinline__ uint32_t dp_probe(uint64_t *word, uint32_t size, uint32_t key, uint32_t r,
                                             uint32_t slot, uint32_t &owner)
{
    const uint64_t mine = ((uint64_t)key << 32) | r;
    for (;;) {
        uint64_t cur = word[slot];
        if (cur == kDpEmpty) {
            cur = atomicCAS(reinterpret_cast<unsigned long long *>(&word[slot]), kDpEmpty, mine);
            if (cur == kDpEmpty) {
                owner = r;
                return slot;  // claimed
            }
        }
        if ((uint32_t)(cur >> 32) == key) {
            owner = (uint32_t)cur;
            return slot;
        }
        slot = dp_next(slot, size);
    }
}

// Full insert from `slot`: probe, confirm an equal key on the 24 bytes, walk
// on past a key collision with a different signature.
__device__ __forceinline__ uint32_t dp_insert(uint64_t *word, uint32_t size, uint32_t key, uint32_t r,
                                              uint32_t slot, const uint8_t *sig, uint32_t stride,
                                              uint32_t &owner)
{
    for (;;) {
        slot = dp_probe(word, size, key, r, slot, owner);
        if (owner == r || sig_equal(sig, stride, r, owner))
            return slot;
        slot = dp_next(slot, size);
    }
}

// LDS table of a partition: 32-bit words {low key bits << kDpLocBits | local
// index of the claimer}.  Within a partition the top d1 + d2 key bits are
// all equal, so the kept 20 bits hold every bit that tells its records apart
// (16 of them at dp_plan's 2^16 partitions for 100M records).
__device__ __forceinline__ uint32_t dp_lprobe(uint32_t *word, uint32_t kb, uint32_t l, uint32_t slot,
                                              uint32_t &owner)
{
    const uint32_t mine = kb << kDpLocBits | l;
    for (;;) {
        uint32_t cur = word[slot];
        if (cur == kDpWEmpty) {
            cur = atomicCAS(&word[slot], kDpWEmpty, mine);
            if (cur == kDpWEmpty) {
                owner = l;
                return slot;  // claimed
            }
        }
        if ((cur >> kDpLocBits) == kb) {
            owner = cur & ((1u << kDpLocBits) - 1);
            return slot;
        }
        slot = dp_next(slot, kDpSlots);
    }
}

// A record's ingest index for the class minimum (only multi-member classes
// read it).  GM_ROW: the 32-byte exchange rows carry it at byte 24, on the
// line the confirmation just read.  GM_REP: from the record's own rep_out
// slot (dp_tile wrote gidx[r] there): the line its final store lands on,
// instead of a third array.  GM_INDEX: no gidx, the record index itself.
enum { GM_INDEX = 0, GM_REP = 1, GM_ROW = 2 };

__device__ __forceinline__ uint64_t gidx_of(const DpOut &out, const uint8_t *sig, uint32_t stride,
                                            int gmode, uint32_t r)
{
    if (gmode == GM_ROW)
        return *reinterpret_cast<const uint64_t *>(sig + (uint64_t)r * stride + 24);
    return gmode == GM_REP ? out.rep_at(r) : (uint64_t)r;
}

// The partition's entries, gathered from its run in each chunk of its
// bucket, in batches of up to kDpRuns runs: rpos[k] = partition-local index
// of run k's first entry, rsrc[k] = ent2 index of local index 0 along run k.
struct DpRuns {
    const uint16_t *cdo;
    uint64_t bs, bsize;
    uint32_t c0, nch, nd2, d;
    __device__ void run(uint32_t k, uint32_t &s, uint32_t &len) const
    {
        const uint16_t *c = cdo + (uint64_t)(c0 + k) * nd2;
        s = c[d];
        const uint64_t rem = bsize - (uint64_t)k * kDpChunk;
        const uint32_t e = d + 1 < nd2 ? c[d + 1] : (uint32_t)(rem < (uint64_t)kDpChunk ? rem : (uint64_t)kDpChunk);
        len = e - s;
    }
};

// Build batch [kb, kb + kDpRuns) starting at local index l0: one scan of
// {s << 32 | len} gives the run positions (low half) and the batch's sums of
// run lengths and of run starts (the entries of the bucket with a smaller
// digit, for the partition's virtual start).  Ends with a barrier.
__device__ __forceinline__ uint64_t dp_batch(const DpRuns &R, uint32_t kb, uint32_t l0, uint32_t *rpos,
                                             uint64_t *rsrc, uint64_t *wsum)
{
    const uint32_t k = kb + threadIdx.x;
    uint32_t s = 0, len = 0;
    if (k < R.nch)
        R.run(k, s, len);
    uint64_t tot;
    const uint64_t ex = block_exclusive_scan64((uint64_t)s << 32 | len, wsum, tot);
    const uint32_t pos = l0 + (uint32_t)ex;
    rpos[threadIdx.x] = pos;
    rsrc[threadIdx.x] = R.bs + (uint64_t)k * kDpChunk + s - pos;
    __syncthreads();
    return tot;
}

// ent2 index of local index l: the last run of the batch starting at or before it.
__device__ __forceinline__ uint64_t dp_src(uint32_t l, uint32_t nk, const uint32_t *rpos, const uint64_t *rsrc)
{
    uint32_t lo = 0, hi = nk;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (rpos[mid] <= l)
            lo = mid;
        else
            hi = mid;
    }
    return rsrc[lo] + l;
}

// Only records of classes with more than one member are written (random
// stores); K1 already wrote every record's singleton answer.  The class
// minimum needs ingest indices only there: every member that joined a
// claimed slot folds min(own, claimer's) into the claimer's minimum, so a
// class of k > 1 members gets all k indices and a singleton reads none.
template <int GM>
using DpMin = typename std::conditional<GM == GM_INDEX, uint32_t, uint64_t>::type;

template <int GM>
struct alignas(16) DpLds {  // 40 KB for GM_INDEX (four workgroups per CU), 48 KB with 64-bit minima
    uint32_t word[kDpSlots + 2];  // the table; before it, the gather's run table (dp_run_tables)
    uint32_t rec[kDpCap];         // local index -> record
    uint32_t cn[kDpCap / 2];      // class sizes (u16 pairs) at the claimer's local index
    uint32_t jl[kDpCap];          // entries that met an equal key: local | claimer << 16; jl[kDpCap - 1] = count
    DpMin<GM> mn[kDpCap];         // class minimum ingest index at the claimer's local index
};
static_assert(sizeof(DpLds<GM_INDEX>) == 40960, "four workgroups per CU");

struct DpArgs {
    const uint64_t *ent2;
    const uint8_t *sig;
    uint32_t stride;
    int gmode;
    uint64_t *gword, *gmin;
    uint32_t *gcnt, *gslot;
    DpOut out;
    DpSink sink;
};

// The gather's run table lives in the LDS table region (dead before the
// table is initialised).
struct DpRunTab {
    uint32_t *rpos;
    uint64_t *rsrc, *wsum;
    template <int GM>
    __device__ explicit DpRunTab(DpLds<GM> &L)
        : rpos(L.word), rsrc(reinterpret_cast<uint64_t *>(L.word + kDpRuns)), wsum(rsrc + kDpRuns)
    {
    }
};
static_assert(kDpRuns + 2 * kDpRuns + 2 * (kDpGroupThreads / 64) <= kDpSlots, "gather tables fit in the table region");

__device__ __forceinline__ void dp_lds_min(uint32_t *p, uint64_t v) { atomicMin(p, (uint32_t)v); }
__device__ __forceinline__ void dp_lds_min(uint64_t *p, uint64_t v)
{
    atomicMin(reinterpret_cast<unsigned long long *>(p), (unsigned long long)v);
}

__device__ __forceinline__ uint32_t dp_cn(const uint32_t *cn, uint32_t l)
{
    return (cn[l >> 1] >> (16 * (l & 1))) & 0xFFFFu;
}

// The LDS grouping of one partition whose key halves and records (kh, rc)
// are in registers, entry k of this thread at local index threadIdx.x + k *
// 512.  Ends with a barrier.
template <int GM>
__device__ __forceinline__ void dp_group_lds(DpLds<GM> &L, const DpArgs &A, const uint32_t (&kh)[kDpEpt],
                                             const uint32_t (&rc)[kDpEpt], uint32_t cnt)
{
    constexpr int NT = kDpGroupThreads;
    for (int k = threadIdx.x; k < (int)kDpSlots; k += NT)
        L.word[k] = kDpWEmpty;
    for (int k = threadIdx.x; k < (int)kDpCap / 2; k += NT)
        L.cn[k] = 0x00010001u;  // every entry counts itself (read at claimers only)
    for (int k = threadIdx.x; k < (int)kDpCap; k += NT)
        L.mn[k] = (DpMin<GM>)~0ull;
#pragma unroll
    for (int k = 0; k < kDpEpt; k++) {
        const uint32_t l = threadIdx.x + k * NT;
        if (l < cnt)
            L.rec[l] = rc[k];
    }
    if (threadIdx.x == 0)
        L.jl[kDpCap - 1] = 0;
    __syncthreads();
    // (1) key-only probes, LDS only; an entry that met an equal key goes to
    // the list (at most cnt - 1 of them: every class has a claimer)
    uint32_t claim = 0;  // bit k: entry k claimed its slot
#pragma unroll
    for (int k = 0; k < kDpEpt; k++) {
        const uint32_t l = threadIdx.x + k * NT;
        if (l < cnt) {
            uint32_t own;
            dp_lprobe(L.word, kh[k] & kDpKeyMask, l, dp_home(kh[k], kDpSlots), own);
            if (own == l)
                claim |= 1u << k;
            else
                L.jl[atomicAdd(&L.jl[kDpCap - 1], 1u)] = l | own << 16;
        }
    }
    __syncthreads();
    // (2) the listed entries confirm on the full 24 bytes -- one per thread
    // for up to 512 of them, both rows' loads in flight together -- and fold
    // into their class
    const uint32_t nj = L.jl[kDpCap - 1];
    for (uint32_t j = threadIdx.x; j < nj; j += NT) {
        const uint32_t e = L.jl[j];
        const uint32_t l = e & 0xFFFFu;
        uint32_t own = e >> 16;
        const uint32_t r = L.rec[l];
        uint32_t o = L.rec[own];
        uint64_t gl = r, go = o;
        uint64_t ra, rb, rcc, oa, ob, oc;
        load_sig(A.sig + (uint64_t)r * A.stride, ra, rb, rcc);
        load_sig(A.sig + (uint64_t)o * A.stride, oa, ob, oc);
        if constexpr (GM != GM_INDEX) {
            gl = gidx_of(A.out, A.sig, A.stride, GM, r);
            go = gidx_of(A.out, A.sig, A.stride, GM, o);
        }
        if (!(ra == oa && rb == ob && rcc == oc)) {
            // a key-bit collision with a different signature (rare):
            // walk on from the slot it met -- the first slot with its
            // key bits along its probe sequence, found again because
            // every slot is set once -- confirming each equal key
            const uint32_t key = (uint32_t)sig_hash(ra, rb, rcc), kb = key & kDpKeyMask;
            uint32_t slot = dp_lprobe(L.word, kb, l, dp_home(key, kDpSlots), own);
            for (;;) {
                slot = dp_lprobe(L.word, kb, l, dp_next(slot, kDpSlots), own);
                if (own == l)
                    break;  // claimed a slot of its own
                o = L.rec[own];
                if (sig_equal(A.sig, A.stride, r, o))
                    break;
            }
            go = GM == GM_INDEX ? (uint64_t)o : gidx_of(A.out, A.sig, A.stride, GM, o);
        }
        if (own != l) {
            atomicAdd(&L.cn[own >> 1], 1u << (16 * (own & 1)));
            dp_lds_min(&L.mn[own], gl < go ? gl : go);
        }
        L.jl[j] = l | own << 16;  // its class (itself if it claimed a slot)
    }
    __syncthreads();
    if (A.sink.ans) {
        // (3') exchange owner: the records of multi-member classes as sink
        // records, counted per segment in LDS (the table's words are dead
        // now), one device-scope atomic per segment this workgroup answers,
        // then placed
        uint32_t *lc = L.word, *lbase = L.word + 64;
        auto each = [&](auto &&f) {
#pragma unroll
            for (int k = 0; k < kDpEpt; k++) {
                const uint32_t l = threadIdx.x + k * NT;
                if ((claim >> k) & 1u) {
                    const uint32_t c = dp_cn(L.cn, l);
                    if (c > 1)
                        f(rc[k], (uint64_t)L.mn[l], c);
                }
            }
            for (uint32_t j = threadIdx.x; j < nj; j += NT) {
                const uint32_t e = L.jl[j];
                const uint32_t own = e >> 16;
                const uint32_t c = dp_cn(L.cn, own);
                if (c > 1)
                    f(L.rec[e & 0xFFFFu], (uint64_t)L.mn[own], c);
            }
        };
        if (threadIdx.x < 64)
            lc[threadIdx.x] = 0;
        __syncthreads();
        each([&](uint32_t r, uint64_t, uint32_t) { atomicAdd(&lc[A.sink.seg_of(r)], 1u); });
        __syncthreads();
        if (threadIdx.x < 64) {
            const uint32_t cnt = lc[threadIdx.x];
            lbase[threadIdx.x] = cnt ? atomicAdd(&A.sink.cntr[threadIdx.x], cnt) : 0u;
            lc[threadIdx.x] = 0;
        }
        __syncthreads();
        each([&](uint32_t r, uint64_t m, uint32_t c) {
            const uint32_t s = A.sink.seg_of(r);
            A.sink.put(s, lbase[s] + atomicAdd(&lc[s], 1u), r, m, c);
        });
        __syncthreads();
        return;
    }
    // (3) answers of the records of multi-member classes
#pragma unroll
    for (int k = 0; k < kDpEpt; k++) {
        const uint32_t l = threadIdx.x + k * NT;
        if ((claim >> k) & 1u) {
            const uint32_t c = dp_cn(L.cn, l);
            if (c > 1) {
                const uint64_t m = L.mn[l];
                // the class's first record keeps dp_tile's rep = r
                A.out.store(rc[k], m, c, GM != GM_INDEX || m != rc[k]);
            }
        }
    }
    for (uint32_t j = threadIdx.x; j < nj; j += NT) {
        const uint32_t e = L.jl[j];
        const uint32_t l = e & 0xFFFFu, own = e >> 16;
        const uint32_t c = dp_cn(L.cn, own);
        if (c > 1) {
            const uint32_t r = L.rec[l];
            const uint64_t m = L.mn[own];
            // with no gidx a listed entry may be its class's first record
            // too (the claimer is whichever entry probed first)
            A.out.store(r, m, c, GM != GM_INDEX || m != r);
        }
    }
    __syncthreads();
}

// A partition's entries as key halves and records (kh, rc), entry k of this
// thread at local index threadIdx.x + k * 512; loads clamped to the last
// entry so that all of a thread's loads leave together.
__device__ __forceinline__ void dp_split_entry(uint64_t en, uint32_t &kh, uint32_t &rc)
{
    kh = (uint32_t)(en >> 32);
    rc = (uint32_t)en;
}

// A partition the pipeline did not gather: a bucket of more than kDpRuns
// chunks (its runs come in batches), or more records than the LDS table
// holds (grouped on a table in its own HBM region, 2 * cnt slots at
// 2 * its virtual start).  Ends with a barrier.
template <int GM>
__device__ __forceinline__ void dp_group_slow(DpLds<GM> &L, const DpArgs &A, const DpRuns &R)
{
    const DpRunTab T(L);
    uint32_t cnt = 0, below = 0;
    for (uint32_t kb = 0; kb < R.nch; kb += kDpRuns) {
        uint32_t s = 0, len = 0;
        if (kb + threadIdx.x < R.nch)
            R.run(kb + threadIdx.x, s, len);
        uint64_t t2;
        block_exclusive_scan64((uint64_t)s << 32 | len, T.wsum, t2);
        cnt += (uint32_t)t2;
        below += (uint32_t)(t2 >> 32);
    }
    if (cnt == 0)
        return;
    if (cnt <= kDpCap) {
        uint32_t kh[kDpEpt], rc[kDpEpt];
#pragma unroll
        for (int k = 0; k < kDpEpt; k++)
            kh[k] = rc[k] = 0;
        for (uint32_t kb = 0, l0 = 0; kb < R.nch; kb += kDpRuns) {
            const uint32_t nk = (R.nch - kb) < (uint32_t)kDpRuns ? (R.nch - kb) : (uint32_t)kDpRuns;
            const uint32_t l1 = l0 + (uint32_t)dp_batch(R, kb, l0, T.rpos, T.rsrc, T.wsum);
#pragma unroll
            for (int k = 0; k < kDpEpt; k++) {
                const uint32_t l = threadIdx.x + k * kDpGroupThreads;
                if (l >= l0 && l < l1)
                    dp_split_entry(A.ent2[dp_src(l, nk, T.rpos, T.rsrc)], kh[k], rc[k]);
            }
            __syncthreads();
            l0 = l1;
        }
        dp_group_lds<GM>(L, A, kh, rc, cnt);
        return;
    }
    const uint64_t vs = R.bs + below;
    const uint32_t size = 2 * cnt;
    uint64_t *w = A.gword + 2ull * vs;
    uint64_t *m = A.gmin + 2ull * vs;
    uint32_t *c = A.gcnt + 2ull * vs;
    for (uint32_t k = threadIdx.x; k < size; k += blockDim.x) {
        w[k] = kDpEmpty;
        m[k] = kDpEmpty;
        c[k] = 0;
    }
    __syncthreads();
    for (uint32_t kb = 0, l0 = 0; kb < R.nch; kb += kDpRuns) {
        const uint32_t nk = (R.nch - kb) < (uint32_t)kDpRuns ? (R.nch - kb) : (uint32_t)kDpRuns;
        const uint32_t l1 = l0 + (uint32_t)dp_batch(R, kb, l0, T.rpos, T.rsrc, T.wsum);
        for (uint32_t l = l0 + threadIdx.x; l < l1; l += blockDim.x) {
            const uint64_t en = A.ent2[dp_src(l, nk, T.rpos, T.rsrc)];
            const uint32_t r = (uint32_t)en, key = (uint32_t)(en >> 32);
            uint32_t o;
            const uint32_t slot = dp_insert(w, size, key, r, dp_home(key, size), A.sig, A.stride, o);
            atomicAdd(&c[slot], 1u);
            if (o != r) {
                const uint64_t a = gidx_of(A.out, A.sig, A.stride, GM, r);
                const uint64_t b2 = gidx_of(A.out, A.sig, A.stride, GM, o);
                atomicMin(reinterpret_cast<unsigned long long *>(&m[slot]), (unsigned long long)(a < b2 ? a : b2));
            }
            A.gslot[vs + l] = slot;
        }
        __syncthreads();
        l0 = l1;
    }
    __threadfence_block();
    __syncthreads();
    for (uint32_t kb = 0, l0 = 0; kb < R.nch; kb += kDpRuns) {
        const uint32_t nk = (R.nch - kb) < (uint32_t)kDpRuns ? (R.nch - kb) : (uint32_t)kDpRuns;
        const uint32_t l1 = l0 + (uint32_t)dp_batch(R, kb, l0, T.rpos, T.rsrc, T.wsum);
        for (uint32_t l = l0 + threadIdx.x; l < l1; l += blockDim.x) {
            const uint32_t slot = A.gslot[vs + l];
            if (c[slot] > 1) {
                const uint32_t r = (uint32_t)A.ent2[dp_src(l, nk, T.rpos, T.rsrc)];
                if (A.sink.ans) {  // rare path: one device-scope atomic per record
                    const uint32_t s = A.sink.seg_of(r);
                    A.sink.put(s, atomicAdd(&A.sink.cntr[s], 1u), r, m[slot], c[slot]);
                } else {
                    A.out.store(r, m[slot], c[slot], true);
                }
            }
        }
        __syncthreads();
        l0 = l1;
    }
}

// K5: one workgroup per partition.  A partition of a bucket with more than
// kDpRuns chunks (its runs come in batches) or of more than kDpCap records
// (the HBM table) is listed for dp_group_slow_kernel instead.
static_assert(kDpRuns == kDpGroupThreads, "one run per thread in a batch");

__device__ __forceinline__ void dp_runs_of(uint32_t q, int d2, uint64_t tiles, const uint64_t *off1,
                                           const uint32_t *cb, const uint16_t *cdo, DpRuns &R)
{
    R.nd2 = 1u << d2;
    R.d = q & (R.nd2 - 1);
    const uint32_t b = q >> d2;
    R.cdo = cdo;
    R.c0 = cb[b];
    R.nch = cb[b + 1] - R.c0;
    R.bs = off1[(uint64_t)b * tiles];
    R.bsize = off1[(uint64_t)(b + 1) * tiles] - R.bs;
}

template <int GM>
__global__ __launch_bounds__(kDpGroupThreads) __attribute__((amdgpu_waves_per_eu(GM == GM_INDEX ? 8 : 6))) void dp_group_kernel(
    const uint64_t *__restrict__ ent2, int d2, uint64_t tiles, const uint64_t *__restrict__ off1,
    const uint32_t *__restrict__ cb, const uint16_t *__restrict__ cdo, const uint8_t *__restrict__ sig,
    uint32_t stride, DpOut out, DpSink sink, uint32_t *__restrict__ slow)
{
    __shared__ DpLds<GM> L;
    const DpRunTab T(L);
    // XCD-aware order: workgroups are dealt to the 8 XCDs round-robin, so
    // XCD x takes a contiguous range of partitions; neighbouring digits of
    // one bucket share the lines of their runs (ent2) and of the chunks'
    // digit starts (cdo) in that XCD's L2 (3.13 against 3.14-3.15 ms per
    // 100M, profiles/r02/dedup_xcd_ab.txt).
    const uint32_t G = gridDim.x, per = G >> 3, rem = G & 7, x = blockIdx.x & 7, i = blockIdx.x >> 3;
    const uint32_t q = x < rem ? x * (per + 1) + i : rem * (per + 1) + (x - rem) * per + i;
    DpRuns R;
    dp_runs_of(q, d2, tiles, off1, cb, cdo, R);
    const uint32_t cnt = R.nch > (uint32_t)kDpRuns ? ~0u : (uint32_t)dp_batch(R, 0, 0, T.rpos, T.rsrc, T.wsum);
    if (cnt == 0)
        return;
    if (cnt > kDpCap) {
        if (threadIdx.x == 0)
            slow[1 + atomicAdd(slow, 1u)] = q;
        return;
    }
    uint32_t kh[kDpEpt], rc[kDpEpt];
#pragma unroll
    for (int k = 0; k < kDpEpt; k++) {
        const uint32_t l = threadIdx.x + k * kDpGroupThreads;
        dp_split_entry(ent2[dp_src(l < cnt ? l : cnt - 1, R.nch, T.rpos, T.rsrc)], kh[k], rc[k]);
    }
    __syncthreads();  // run table reads done before the table init
    const DpArgs A{ent2, sig, stride, GM, nullptr, nullptr, nullptr, nullptr, out, sink};
    dp_group_lds<GM>(L, A, kh, rc, cnt);
}

// The listed partitions (slow[0] of them), a few persistent workgroups.
template <int GM>
__global__ __launch_bounds__(kDpGroupThreads) void dp_group_slow_kernel(
    const uint64_t *__restrict__ ent2, int d2, uint64_t tiles, const uint64_t *__restrict__ off1,
    const uint32_t *__restrict__ cb, const uint16_t *__restrict__ cdo, const uint8_t *__restrict__ sig,
    uint32_t stride, uint64_t *__restrict__ gword, uint64_t *__restrict__ gmin,
    uint32_t *__restrict__ gcnt, uint32_t *__restrict__ gslot, DpOut out, DpSink sink,
    const uint32_t *__restrict__ slow)
{
    __shared__ DpLds<GM> L;
    const DpArgs A{ent2, sig, stride, GM, gword, gmin, gcnt, gslot, out, sink};
    const uint32_t ns = slow[0];
    for (uint32_t i = blockIdx.x; i < ns; i += gridDim.x) {
        DpRuns R;
        dp_runs_of(slow[1 + i], d2, tiles, off1, cb, cdo, R);
        dp_group_slow<GM>(L, A, R);
        __syncthreads();
    }
}

// Workspace layout of launch_dedup_group (bytes, 256-aligned pieces).
static inline uint64_t al(uint64_t x) { return (x + 255) & ~255ull; }

uint64_t dedup_ws_bytes(uint64_t n)
{
    const DpPlan pl = dp_plan(n);
    const uint64_t ncnt = pl.ncnt();
    return al(8 * n) + al(8 * n) + al(8 * (ncnt + 1)) + al(8 * (ncnt + 1)) + al(8 * scan_workspace_elems(ncnt)) +
           al(4 * ncnt) + al(4 * ((1ull << pl.d1) + 1)) + al(4 * pl.chunks) + al(16 * pl.chunks) +
           al((2 * pl.chunks) << pl.d2) +
           al(16 * n) + al(16 * n) + al(8 * n) + al(4 * (pl.nparts() + 1));
}

static unsigned grid_for(uint64_t n, unsigned block)
{
    uint64_t g = (n + block - 1) / block;
    if (g > 16384)
        g = 16384;
    return g ? (unsigned)g : 1u;
}

hipError_t launch_dedup_group(const uint8_t *sig, uint32_t sig_stride, const uint64_t *gidx,
                              uint32_t gidx_stride, uint64_t n, void *ws, uint64_t *rep_out,
                              uint32_t *ref_out, bool packed, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1,
                              const DedupSink *xs)
{
    if (n == 0)
        return hipSuccess;
    const DpPlan pl = dp_plan(n);
    const uint64_t ncnt = pl.ncnt();
    char *p = static_cast<char *>(ws);
    auto take = [&](uint64_t bytes) {
        char *q = p;
        p += al(bytes);
        return q;
    };
    uint64_t *ent1 = reinterpret_cast<uint64_t *>(take(8 * n));
    uint64_t *ent2 = reinterpret_cast<uint64_t *>(take(8 * n));
    uint64_t *cnt1 = reinterpret_cast<uint64_t *>(take(8 * (ncnt + 1)));
    uint64_t *off1 = reinterpret_cast<uint64_t *>(take(8 * (ncnt + 1)));
    uint64_t *bsum = reinterpret_cast<uint64_t *>(take(8 * scan_workspace_elems(ncnt)));
    uint32_t *loc1 = reinterpret_cast<uint32_t *>(take(4 * ncnt));
    uint32_t *cb = reinterpret_cast<uint32_t *>(take(4 * ((1ull << pl.d1) + 1)));
    uint32_t *chunk_ta = reinterpret_cast<uint32_t *>(take(4 * pl.chunks));
    uint4 *chunk_hd = reinterpret_cast<uint4 *>(take(16 * pl.chunks));
    uint16_t *cdo = reinterpret_cast<uint16_t *>(take((2 * pl.chunks) << pl.d2));
    uint64_t *gword = reinterpret_cast<uint64_t *>(take(16 * n));  // oversized-partition tables
    uint64_t *gmin = reinterpret_cast<uint64_t *>(take(16 * n));
    uint32_t *gcnt = reinterpret_cast<uint32_t *>(take(8 * n));
    uint32_t *slow = reinterpret_cast<uint32_t *>(take(4 * (pl.nparts() + 1)));  // count, partitions
    uint32_t *gslot = reinterpret_cast<uint32_t *>(ent1);  // ent1 is dead after dp_split
    // with a sink the answers go there (multi-member classes only) and no
    // singleton answer is written (dp_tile skips its stores)
    const DpOut out{xs ? nullptr : rep_out, xs ? nullptr : ref_out, packed};
    DpSink sink{nullptr, nullptr, nullptr, 0};
    if (xs)
        sink = DpSink{static_cast<uint4 *>(xs->ans), xs->cntr, xs->seg, xs->nseg};
    hipError_t e;
    if (ev0)
        (void)hipEventRecord(ev0, st);
    dp_tile_kernel<<<(unsigned)pl.tiles, kDpTileThreads, 0, st>>>(sig, sig_stride, gidx, gidx_stride, n, pl.d1,
                                                                  pl.tiles, ent1, out, cnt1, loc1);
    if ((e = launch_exclusive_scan(cnt1, ncnt, off1, bsum, st)) != hipSuccess)
        return e;
    dp_chunks_kernel<<<1, 256, 0, st>>>(off1, pl.d1, pl.tiles, cb, slow);
    dp_chunk_ta_kernel<<<grid_for(ncnt, 256), 256, 0, st>>>(off1, pl.tiles, ncnt, cb, chunk_ta, chunk_hd);
#define DP_SPLIT(NB)                                                                                     \
    dp_split_kernel<NB><<<(unsigned)pl.chunks, kDpSplitThreads, 0, st>>>(                                \
        ent1, pl.d1, pl.d2, pl.tiles, off1, loc1, cb, chunk_ta, chunk_hd, ent2, cdo, out, gidx, gidx_stride, n)
    if (pl.d2 <= 10)
        DP_SPLIT(1024);
    else
        DP_SPLIT(1 << kDpMaxD2);
#undef DP_SPLIT
    const int gmode = !gidx_stride ? GM_INDEX
                      : (gidx == reinterpret_cast<const uint64_t *>(sig + 24) && 8 * gidx_stride == sig_stride)
                          ? GM_ROW
                          : GM_REP;
#define DP_GROUP(G)                                                                                       \
    dp_group_kernel<G><<<(unsigned)pl.nparts(), kDpGroupThreads, 0, st>>>(ent2, pl.d2, pl.tiles, off1, cb, cdo, sig, \
                                                                        sig_stride, out, sink, slow)
    if (gmode == GM_ROW)
        DP_GROUP(GM_ROW);
    else if (gmode == GM_REP)
        DP_GROUP(GM_REP);
    else
        DP_GROUP(GM_INDEX);
#undef DP_GROUP
    if (gmode == GM_ROW)
        dp_group_slow_kernel<GM_ROW><<<256, kDpGroupThreads, 0, st>>>(ent2, pl.d2, pl.tiles, off1, cb, cdo, sig,
                                                                    sig_stride, gword, gmin, gcnt, gslot, out, sink, slow);
    else if (gmode == GM_REP)
        dp_group_slow_kernel<GM_REP><<<256, kDpGroupThreads, 0, st>>>(ent2, pl.d2, pl.tiles, off1, cb, cdo, sig,
                                                                    sig_stride, gword, gmin, gcnt, gslot, out, sink, slow);
    else
        dp_group_slow_kernel<GM_INDEX><<<256, kDpGroupThreads, 0, st>>>(ent2, pl.d2, pl.tiles, off1, cb, cdo, sig,
                                                                      sig_stride, gword, gmin, gcnt, gslot, out, sink, slow);
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

// Bucketing by owner in tiles of kBkTile records, with no device-scope
// atomics: bucket_count_kernel writes each tile's count per owner
// (cnt[owner * tiles + tile]), one exclusive scan of those gives where every
// (owner, tile) run starts in the owner-grouped rows (owner-major, so each
// owner's rows are contiguous), and bucket_scatter_kernel places each tile's
// records at their run's start plus their rank among the tile's records of
// that owner (an LDS counter).  Round 4's form (every block of 256 records
// reserving its ranges with one global atomic per owner on shared cursors,
// and summing its counts the same way) spent 0.81 ms per 12.5M records in
// those atomics (profiles/r05/dedup_rank_share.txt); this form reads the
// signatures twice and writes each row once.
constexpr int kBkThreads = 256, kBkItems = 32, kBkTile = kBkThreads * kBkItems;  // 8192: one-block scan up to 16K (owner, tile) counts

uint64_t bucket_tiles(uint64_t n) { return (n + kBkTile - 1) / kBkTile; }

size_t bucket_ws_elems(uint64_t n)  // u64 words: cnt and off (64 owners x tiles + 1 each), the scan's block sums
{
    const uint64_t nt = 64 * bucket_tiles(n) + 1;
    return 2 * nt + scan_workspace_elems(nt) + 2;
}

__global__ __launch_bounds__(kBkThreads) void bucket_count_kernel(const uint8_t *__restrict__ sig, uint64_t n,
                                                                  uint32_t nranks, uint64_t tiles,
                                                                  uint64_t *__restrict__ cnt)
{
    __shared__ uint32_t h[kBkThreads / 64][64];  // per wave: fewer lanes on one LDS counter
    const int w = threadIdx.x >> 6;
    for (int k = threadIdx.x; k < (kBkThreads / 64) * 64; k += kBkThreads)
        (&h[0][0])[k] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kBkTile;
#pragma unroll 4
    for (int it = 0; it < kBkItems; it++) {
        const uint64_t r = t0 + (uint64_t)it * kBkThreads + threadIdx.x;
        if (r < n)
            atomicAdd(&h[w][owner_of(sig + 24 * r, nranks)], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nranks; k += kBkThreads) {
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < kBkThreads / 64; q++)
            c += h[q][k];
        cnt[(uint64_t)k * tiles + blockIdx.x] = c;
    }
}

// off: the scan of cnt (off[nranks * tiles] = n).  Block 0 also writes each
// owner's row count (counts_out[q], the announcement's first nranks words).
// x (fdfs_gpu_dedup_global, round 6): the rank's own rows (owner x.me) go
// straight to the front of its owner-side receive buffer (x.self_rows: no
// self copy), rec_of[send position] = record (the owner answers by send
// position), and every record's singleton answer (rep = gidx, ref = 1) is
// written here, coalesced, so that the owners return only the records of
// multi-member classes.
__global__ __launch_bounds__(kBkThreads) void bucket_scatter_kernel(
    const uint8_t *__restrict__ sig, const uint64_t *__restrict__ gidx, uint64_t n, uint32_t nranks,
    uint64_t tiles, const uint64_t *__restrict__ off, uint8_t *__restrict__ rows, uint64_t *__restrict__ row_of,
    uint64_t *__restrict__ counts_out, BucketExtra x)
{
    __shared__ uint32_t cnt[64];
    __shared__ uint64_t bas[64];
    if (threadIdx.x < nranks) {
        cnt[threadIdx.x] = 0;
        bas[threadIdx.x] = off[(uint64_t)threadIdx.x * tiles + blockIdx.x];
        if (blockIdx.x == 0)
            counts_out[threadIdx.x] = off[(uint64_t)(threadIdx.x + 1) * tiles] - off[(uint64_t)threadIdx.x * tiles];
    }
    __syncthreads();
    const uint64_t self0 = x.self_rows ? off[(uint64_t)x.me * tiles] : 0;  // the own segment's first send position
    const uint64_t t0 = (uint64_t)blockIdx.x * kBkTile;
#pragma unroll 4
    for (int it = 0; it < kBkItems; it++) {
        const uint64_t r = t0 + (uint64_t)it * kBkThreads + threadIdx.x;
        if (r < n) {
            uint64_t a, b, c;
            load_sig(sig + 24 * r, a, b, c);
            const uint32_t own = (uint32_t)((sig_hash(a, b, c) >> 32) % nranks);  // owner_of
            const uint64_t pos = bas[own] + atomicAdd(&cnt[own], 1u);
            const uint64_t g = gidx ? gidx[r] : r;
            uint8_t *dst = (x.self_rows && own == x.me) ? x.self_rows + 32 * (pos - self0) : rows + 32 * pos;
            uint4 *d = reinterpret_cast<uint4 *>(dst);  // two 16-byte stores per row
            d[0] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
            d[1] = make_uint4((uint32_t)c, (uint32_t)(c >> 32), (uint32_t)g, (uint32_t)(g >> 32));
            if (row_of)
                row_of[r] = pos;
            if (x.rec_of)
                x.rec_of[pos] = (uint32_t)r;
            if (x.rep_out) {
                x.rep_out[r] = g;
                x.ref_out[r] = 1u;
            }
        }
    }
}

// fdfs_gpu_dedup_global's bucket in one pass (round 6): owner q's rows go to
// a fixed-capacity region [q cap, q cap + cnt_q) of the send order, and each
// tile reserves its per-owner ranges with one device-scope atomic per owner
// on the announcement's count words (12.5M records: ~3K tiles x 8 owners,
// against round 4's 390K per-block atomics) -- no counting pass over the
// signatures and no scan.  A tile's records stay in registers between the
// LDS count (per wave, the atomic's return is the record's rank) and the
// stores, so each signature is read once.  cap = n / nranks plus slack
// (bucket_cap); an owner count above it (skewed owners: one signature
// repeated many times) is not written, and every rank sees it in the
// all-gathered counts and buckets again with the exact two-pass form.
constexpr int kBpItems = 16, kBpTile = kBkThreads * kBpItems;  // 4096 records per tile

uint64_t bucket_cap(uint64_t n, uint32_t nranks)
{
    if (nranks <= 1)
        return n;
    const uint64_t mean = (n + nranks - 1) / nranks;
    uint64_t sd = 1;
    while (sd * sd < mean)
        sd++;
    const uint64_t cap = mean + 8 * sd + 1024;  // binomial owner counts: 8 sigma
    return cap < n ? cap : n;
}

__global__ __launch_bounds__(kBkThreads) void bucket_place_kernel(
    const uint8_t *__restrict__ sig, const uint64_t *__restrict__ gidx, uint64_t n, uint32_t nranks, uint64_t cap,
    uint8_t *__restrict__ rows, unsigned long long *__restrict__ counts, BucketExtra x)
{
    __shared__ uint32_t h[kBkThreads / 64][64];  // per wave: fewer lanes on one LDS counter
    __shared__ uint64_t wb[kBkThreads / 64][64];  // the wave's first slot per owner
    const int w = threadIdx.x >> 6;
    for (int k = threadIdx.x; k < (kBkThreads / 64) * 64; k += kBkThreads)
        (&h[0][0])[k] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kBpTile;
    uint64_t a[kBpItems], b[kBpItems], c[kBpItems];
    uint32_t ok[kBpItems];  // owner << 16 | rank among the wave's records of that owner
#pragma unroll
    for (int it = 0; it < kBpItems; it++) {
        const uint64_t r = t0 + (uint64_t)it * kBkThreads + threadIdx.x;
        a[it] = b[it] = c[it] = 0;
        ok[it] = 0;
        if (r < n) {
            load_sig(sig + 24 * r, a[it], b[it], c[it]);
            const uint32_t own = (uint32_t)((sig_hash(a[it], b[it], c[it]) >> 32) % nranks);  // owner_of
            ok[it] = own << 16 | atomicAdd(&h[w][own], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < nranks) {
        const uint32_t q = threadIdx.x;
        uint32_t tot = 0;
#pragma unroll
        for (int v = 0; v < kBkThreads / 64; v++)
            tot += h[v][q];
        uint64_t base = tot ? (uint64_t)atomicAdd(&counts[q], (unsigned long long)tot) : 0;
#pragma unroll
        for (int v = 0; v < kBkThreads / 64; v++) {
            wb[v][q] = base;
            base += h[v][q];
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kBpItems; it++) {
        const uint64_t r = t0 + (uint64_t)it * kBkThreads + threadIdx.x;
        if (r < n) {
            const uint32_t own = ok[it] >> 16;
            const uint64_t k = wb[w][own] + (ok[it] & 0xFFFFu);
            const uint64_t g = gidx ? gidx[r] : r;
            if (k < cap) {
                const uint64_t pos = (uint64_t)own * cap + k;
                uint8_t *dst = (x.self_rows && own == x.me) ? x.self_rows + 32 * k : rows + 32 * pos;
                uint4 *d = reinterpret_cast<uint4 *>(dst);
                d[0] = make_uint4((uint32_t)a[it], (uint32_t)(a[it] >> 32), (uint32_t)b[it], (uint32_t)(b[it] >> 32));
                d[1] = make_uint4((uint32_t)c[it], (uint32_t)(c[it] >> 32), (uint32_t)g, (uint32_t)(g >> 32));
                x.rec_of[pos] = (uint32_t)r;
            }
            x.rep_out[r] = g;
            x.ref_out[r] = 1u;
        }
    }
}

hipError_t launch_bucket_place(const uint8_t *sig, const uint64_t *gidx, uint64_t n, uint32_t nranks,
                               uint64_t cap, uint8_t *rows, uint64_t *counts, const BucketExtra &x, hipStream_t st,
                               hipEvent_t ev0, hipEvent_t ev1)
{
    hipError_t e = launch_zero_u32(counts, 2ull * nranks, st);
    if (e != hipSuccess)
        return e;
    if (ev0)
        (void)hipEventRecord(ev0, st);
    if (n)
        bucket_place_kernel<<<(unsigned)((n + kBpTile - 1) / kBpTile), kBkThreads, 0, st>>>(
            sig, gidx, n, nranks, cap, rows, reinterpret_cast<unsigned long long *>(counts), x);
    if (ev1)
        (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

// Multi-GPU dedup (fdfs_gpu_dedup_global): the exchanged {rep, ref} answers
// (the owners' packed group output) mapped back to the rank's records
// through row_of.  (The torch-form exchange of fastdfs_amd/dist.py routes
// answers this way; the C ABI's own exchange applies sink records instead.)
__global__ void answer_gather_kernel(const uint64_t *__restrict__ back, const uint64_t *__restrict__ row_of,
                                     uint64_t n, uint64_t *__restrict__ rep_out, uint32_t *__restrict__ ref_out)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const ulonglong2 a = reinterpret_cast<const ulonglong2 *>(back)[row_of[i]];
        rep_out[i] = a.x;
        ref_out[i] = (uint32_t)a.y;
    }
}

hipError_t launch_answer_gather(const uint64_t *back, const uint64_t *row_of, uint64_t n, uint64_t *rep_out,
                                uint32_t *ref_out, hipStream_t st)
{
    if (n)
        answer_gather_kernel<<<grid_for(n, 256), 256, 0, st>>>(back, row_of, n, rep_out, ref_out);
    return hipGetLastError();
}

// Owner q's segment table from the all-gathered announcements (ann: rank p's
// row counts per owner at ann[p * w + q], its cap at ann[p * w + nranks + 3]):
// segment k of q's received rows
// holds the rows of rank dg_seg_src(q, k) (its own first), seg[k] = its first
// row, seg[kSinkSoff + k] = where those rows start in their sender's send
// order; the per-segment sink counters zeroed.  One thread: <= 64 ranks.
__global__ void sink_plan_kernel(const uint64_t *__restrict__ ann, uint32_t w, uint32_t nranks, uint32_t q,
                                 bool exact, uint64_t *__restrict__ seg, uint32_t *__restrict__ cntr)
{
    if (threadIdx.x < 64)
        cntr[threadIdx.x] = 0;
    if (threadIdx.x != 0)
        return;
    uint64_t start = 0;
    for (uint32_t k = 0; k < nranks; k++) {
        const uint32_t p = dg_seg_src(q, k);
        // the sender's layout: fixed-capacity owner regions (its announced
        // cap, launch_bucket_place) or, after a rebucket, the exact prefix
        const uint64_t cap = exact ? 0 : ann[(uint64_t)p * w + nranks + 3];
        uint64_t soff = 0;
        if (cap)
            soff = (uint64_t)q * cap;
        else
            for (uint32_t j = 0; j < q; j++)
                soff += ann[(uint64_t)p * w + j];
        seg[k] = start;
        seg[kSinkSoff + k] = soff;
        start += ann[(uint64_t)p * w + q];
    }
    seg[nranks] = start;
}

hipError_t launch_sink_plan(const uint64_t *ann, uint32_t w, uint32_t nranks, uint32_t q, bool exact, uint64_t *seg,
                            uint32_t *cntr, hipStream_t st)
{
    sink_plan_kernel<<<1, 64, 0, st>>>(ann, w, nranks, q, exact, seg, cntr);
    return hipGetLastError();
}

// The sink records that reached this rank, applied over its pre-filled
// singleton answers: list a (count on the device: its own segment's, still
// in its owner-side buffer) and list b (count known on the host: the other
// owners' records after the way back).
__global__ void answer_apply_kernel(const uint4 *__restrict__ a, const uint32_t *__restrict__ na,
                                    const uint4 *__restrict__ b, uint64_t nb, const uint32_t *__restrict__ rec_of,
                                    uint64_t *__restrict__ rep_out, uint32_t *__restrict__ ref_out)
{
    const uint64_t n1 = na ? *na : 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n1 + nb;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = i < n1 ? a[i] : b[i - n1];
        const uint32_t r = rec_of[v.x];
        rep_out[r] = (uint64_t)v.w << 32 | v.z;
        ref_out[r] = v.y;
    }
}

hipError_t launch_answer_apply(const void *a, const uint32_t *na, uint64_t na_max, const void *b, uint64_t nb,
                               const uint32_t *rec_of, uint64_t *rep_out, uint32_t *ref_out, hipStream_t st)
{
    if (na_max + nb)
        answer_apply_kernel<<<grid_for(na_max + nb, 256), 256, 0, st>>>(
            static_cast<const uint4 *>(a), na, static_cast<const uint4 *>(b), nb, rec_of, rep_out, ref_out);
    return hipGetLastError();
}

hipError_t launch_dedup_bucket(const uint8_t *sig, const uint64_t *gidx, uint64_t n,
                               uint32_t nranks, uint8_t *records_out, uint64_t *counts_out,
                               uint64_t *ws, uint64_t *row_of_out, hipStream_t st,
                               hipEvent_t ev0, hipEvent_t ev1, const BucketExtra *extra)
{
    const BucketExtra x = extra ? *extra : BucketExtra{0, nullptr, nullptr, nullptr, nullptr};
    hipError_t e;
    if (n == 0)
        return launch_zero_u32(counts_out, 2ull * nranks, st);
    const uint64_t tiles = bucket_tiles(n), nt = (uint64_t)nranks * tiles;
    uint64_t *cnt = ws, *off = ws + 64 * tiles + 1, *bsum = off + 64 * tiles + 1;
    if (ev0)
        (void)hipEventRecord(ev0, st);
    bucket_count_kernel<<<(unsigned)tiles, kBkThreads, 0, st>>>(sig, n, nranks, tiles, cnt);
    if ((e = launch_exclusive_scan(cnt, nt, off, bsum, st)) != hipSuccess)
        return e;
    bucket_scatter_kernel<<<(unsigned)tiles, kBkThreads, 0, st>>>(sig, gidx, n, nranks, tiles, off, records_out,
                                                                  row_of_out, counts_out, x);
    if (ev1)
        (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

}  // namespace fdfs
